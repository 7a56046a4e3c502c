// k8s.cpp — resource.Quantity parsing (UP k8s.io/apimachinery/pkg/api/resource/quantity.go#
// ParseQuantity, Quantity.MilliValue, Quantity.Value): exact rational arithmetic, values round up
// (ScaledValue semantics), so "0.1m" cpu is 1 millicore and "1.5Ki" memory is 1536 bytes.
#include "k8s.hpp"

#include <cctype>

namespace qsfw {
namespace {

using i128 = __int128;

struct Rational {
    i128 num, den;  // value = num / den, den > 0
};

i128 checked_mul(i128 a, i128 b, const std::string &s) {
    i128 r;
    if (__builtin_mul_overflow(a, b, &r)) throw QuantityError("quantity: out of range in '" + s + "'");
    return r;
}

Rational parse(const std::string &s) {
    size_t i = 0;
    bool neg = false;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
    i128 mant = 0, den = 1;
    int digits = 0;
    bool seen_point = false;
    for (; i < s.size(); ++i) {
        const char ch = s[i];
        if (ch == '.') {
            if (seen_point) throw QuantityError("quantity: two decimal points in '" + s + "'");
            seen_point = true;
            continue;
        }
        if (!std::isdigit((unsigned char)ch)) break;
        if (++digits > 30) throw QuantityError("quantity: too many digits in '" + s + "'");
        mant = mant * 10 + (ch - '0');
        if (seen_point) den *= 10;
    }
    if (digits == 0) throw QuantityError("quantity: no digits in '" + s + "'");
    const std::string suf = s.substr(i);
    i128 mul = 1, div = 1;
    auto pow10 = [](int e) { i128 v = 1; while (e-- > 0) v *= 10; return v; };
    static const std::map<std::string, int> bin = {{"Ki", 10}, {"Mi", 20}, {"Gi", 30}, {"Ti", 40}, {"Pi", 50}, {"Ei", 60}};
    static const std::map<std::string, int> dec = {{"n", -9}, {"u", -6}, {"m", -3}, {"", 0}, {"k", 3},
                                                    {"M", 6}, {"G", 9}, {"T", 12}, {"P", 15}, {"E", 18}};
    if (auto b = bin.find(suf); b != bin.end()) {
        mul = (i128)1 << b->second;
    } else if (auto d = dec.find(suf); d != dec.end()) {
        if (d->second >= 0) mul = pow10(d->second); else div = pow10(-d->second);
    } else if (!suf.empty() && (suf[0] == 'e' || suf[0] == 'E')) {
        size_t j = 1;
        bool eneg = false;
        if (j < suf.size() && (suf[j] == '+' || suf[j] == '-')) eneg = suf[j++] == '-';
        if (j >= suf.size()) throw QuantityError("quantity: bad exponent in '" + s + "'");
        int e = 0;
        for (; j < suf.size(); ++j) {
            if (!std::isdigit((unsigned char)suf[j])) throw QuantityError("quantity: bad exponent in '" + s + "'");
            e = e * 10 + (suf[j] - '0');
            if (e > 18) throw QuantityError("quantity: exponent out of range in '" + s + "'");
        }
        if (eneg) div = pow10(e); else mul = pow10(e);
    } else {
        throw QuantityError("quantity: unknown suffix '" + suf + "' in '" + s + "'");
    }
    // 30 digits (< 2^100) times a suffix factor up to 2^60 / 10^18 can leave the i128 range:
    // checked, so an absurd quantity is a QuantityError rather than signed overflow
    Rational r{checked_mul(mant, mul, s), checked_mul(den, div, s)};
    if (neg) r.num = -r.num;
    return r;
}

int64_t ceil_div(i128 num, i128 den) {
    if (den <= 0) throw QuantityError("quantity: bad denominator");
    i128 q = num / den;
    if (num % den != 0 && num > 0) ++q;
    if (q > (i128)INT64_MAX || q < (i128)INT64_MIN) throw QuantityError("quantity: out of int64 range");
    return (int64_t)q;
}

}  // namespace

int64_t parse_quantity_milli(const std::string &s) {
    const Rational r = parse(s);
    return ceil_div(checked_mul(r.num, 1000, s), r.den);
}

int64_t value(const std::string &s) {
    const Rational r = parse(s);
    return ceil_div(r.num, r.den);
}

}  // namespace qsfw
