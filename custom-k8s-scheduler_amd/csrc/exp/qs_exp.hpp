// qs_exp.hpp — timing-ablation variants of the resident resolver, force-included
// only by `make exp` (tools/exp_run.sh).  Every variant gives WRONG placements by construction: they
// measure how much of a step the key arithmetic / the parked waves cost.  Never part of libqsched.so.
//   -DQS_EXP_PLAIN_AB  waves A / B take the plain (non-normalizing) slot-key path
//   -DQS_EXP_CHEAP_AB  waves A / B: no key arithmetic (a trivial key from the row)
//   -DQS_EXP_CHEAP_C   wave C: no key arithmetic for its candidate
//   -DQS_EXP_NOPARK    the parked waves skip their per-step statics work
#pragma once
#define QS_EXP_HOOKS 1

#ifdef QS_EXP_PLAIN_AB
#define QS_EXP_NORM_AB(norm) false
#else
#define QS_EXP_NORM_AB(norm) (norm)
#endif

#ifdef QS_EXP_CHEAP_AB
#define QS_EXP_SLOT_KEY(act, r, q) return (act) ? ((uint64_t)(((uint32_t)((r).rc + (q).rc) & 511u) + 1) << 32) : 0ull;
#else
#define QS_EXP_SLOT_KEY(act, r, q)
#endif

#ifdef QS_EXP_CHEAP_C
#define QS_EXP_CAND_KEY(f, tot, cr, p) \
    f = true;                          \
    tot = (uint32_t)((cr).rc + (p).rc) & 511u;
#else
#define QS_EXP_CAND_KEY(f, tot, cr, p)
#endif

#ifdef QS_EXP_NOPARK
#define QS_EXP_PARK_RETURN() return;
#else
#define QS_EXP_PARK_RETURN()
#endif
