// test_framework.cpp — table-driven tests of the C++ framework layer (custom-k8s-scheduler_amd/host)
// in the style of upstream's plugin tests (UP pkg/scheduler/framework/plugins/{noderesources/
// fit_test.go, least_allocated_test.go, balanced_allocation_test.go, tainttoleration/
// taint_toleration_test.go, nodeaffinity/node_affinity_test.go}, UP core/v1/toleration_test.go):
// pods and nodes are built with MakePod / MakeNode, expected scores are recomputed by hand from
// spec/semantics.md (the reference holds no fixtures: parity unpinned).
//
//   test_framework --cpu   host logic only (quantities, interning, pod requests, QoS sort, FitError)
//                          and the CPU reference plugins (host/cpu_plugins.cpp): scores vs the
//                          oracle's scorers, and whole ScheduleOne loops vs the oracle
//   test_framework --gpu   the QoSGPU plugins on the device: filter/score tables, and the whole
//                          ScheduleOne loop on a config-4 cluster built from k8s objects, checked
//                          pod-by-pod against qs_schedule_stream and the CPU oracle.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../custom-k8s-scheduler_amd/host/cpu_plugins.hpp"
#include "../../custom-k8s-scheduler_amd/host/qos_gpu.hpp"
#include "../../tools/oracle_cfg.hpp"
#include "../../tools/synth_objects.hpp"
extern "C" {
#include "../../oracle/qs_oracle.h"
}

using namespace qsfw;

static int g_fail = 0, g_checks = 0;
#define CHECK(c)                                                                   \
    do {                                                                           \
        ++g_checks;                                                                \
        if (!(c)) {                                                                \
            ++g_fail;                                                              \
            std::fprintf(stderr, "  FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);     \
        }                                                                          \
    } while (0)
#define CHECK_EQ(a, b)                                                                         \
    do {                                                                                       \
        ++g_checks;                                                                            \
        auto va_ = (a);                                                                        \
        auto vb_ = (b);                                                                        \
        if (!(va_ == vb_)) {                                                                   \
            ++g_fail;                                                                          \
            std::fprintf(stderr, "  FAIL %s:%d: %s == %s (%s vs %s)\n", __FILE__, __LINE__, #a, \
                         #b, to_s(va_).c_str(), to_s(vb_).c_str());                            \
        }                                                                                      \
    } while (0)
[[maybe_unused]] static std::string to_s(long long v) { return std::to_string(v); }
[[maybe_unused]] static std::string to_s(long v) { return std::to_string(v); }
[[maybe_unused]] static std::string to_s(unsigned long long v) { return std::to_string(v); }
[[maybe_unused]] static std::string to_s(unsigned long v) { return std::to_string(v); }
[[maybe_unused]] static std::string to_s(int v) { return std::to_string(v); }
[[maybe_unused]] static std::string to_s(bool v) { return v ? "true" : "false"; }
[[maybe_unused]] static std::string to_s(const std::string &v) { return '"' + v + '"'; }
[[maybe_unused]] static std::string to_s(Code c) { return std::to_string((int)c); }

struct Case {
    const char *name;
    std::function<void()> fn;
};

// =============================================================================================
// host-only tests
// =============================================================================================
static void test_quantity() {
    struct Q { const char *s; int64_t milli, value; } qs[] = {
        {"500m", 500, 1}, {"1", 1000, 1}, {"1.5", 1500, 2}, {"0.1m", 1, 1}, {"2Gi", 2147483648000LL, 2147483648LL},
        {"1Ki", 1024000, 1024}, {"1.5Gi", 1610612736000LL, 1610612736LL}, {"100M", 100000000000LL, 100000000},
        {"1e3", 1000000, 1000}, {"128Mi", 134217728000LL, 134217728}, {"0", 0, 0}, {"250u", 1, 1}};
    for (const auto &q : qs) {
        CHECK_EQ(parse_quantity_milli(q.s), q.milli);
        CHECK_EQ(value(q.s), q.value);
    }
    for (const char *bad : {"", "abc", "1Qi", "1.2.3", "e3", "1e"}) {
        bool threw = false;
        try { (void)value(bad); } catch (const QuantityError &) { threw = true; }
        CHECK(threw);
    }
}

static void test_tolerations() {
    // UP core/v1/toleration_test.go#TestTolerationToleratesTaint (shape)
    const Taint t{"foo", "bar", kNoSchedule};
    struct C { Toleration tol; bool want; } cs[] = {
        {{"", "Exists", "", ""}, true},                 // empty key + Exists tolerates everything
        {{"foo", "Exists", "", ""}, true},
        {{"foo", "Equal", "bar", kNoSchedule}, true},
        {{"foo", "Equal", "baz", kNoSchedule}, false},  // value mismatch
        {{"foo", "Equal", "bar", kNoExecute}, false},   // effect mismatch
        {{"foo", "", "bar", ""}, true},                 // "" operator means Equal
        {{"other", "Exists", "", ""}, false},
    };
    for (const auto &c : cs) CHECK_EQ(tolerates(c.tol, t), c.want);
}

static void test_requirements() {
    const std::map<std::string, std::string> lb = {{"zone", "z1"}, {"size", "8"}, {"ssd", "true"}};
    struct C { NodeSelectorRequirement r; bool want; } cs[] = {
        {{"zone", "In", {"z1", "z2"}}, true},   {{"zone", "In", {"z3"}}, false},
        {{"zone", "NotIn", {"z3"}}, true},      {{"rack", "NotIn", {"r1"}}, true},
        {{"zone", "NotIn", {"z1"}}, false},     {{"ssd", "Exists", {}}, true},
        {{"gpu", "Exists", {}}, false},         {{"gpu", "DoesNotExist", {}}, true},
        {{"size", "Gt", {"4"}}, true},          {{"size", "Gt", {"8"}}, false},
        {{"size", "Lt", {"16"}}, true},         {{"zone", "Gt", {"1"}}, false},  // non-integer label
        {{"size", "Gt", {"a"}}, false},         {{"zone", "In", {}}, false},     // invalid: no values
    };
    for (const auto &c : cs) CHECK_EQ(requirement_matches(c.r, lb), c.want);
}

static void test_interner() {
    Interner in;
    const Node n = MakeNode("n").Label("zone", "z1").Label("pool", "gpu")
                       .Taint("gpu", "true", kNoSchedule).Taint("maint", "true", kPreferNoSchedule).Obj();
    uint64_t th, ts, lb[2];
    in.node_masks(n, &th, &ts, lb);
    CHECK_EQ(th, (uint64_t)1);  // gpu -> bit 0
    CHECK_EQ(ts, (uint64_t)2);  // maint -> bit 1
    qs_pod rec{};
    // tolerates gpu (NoSchedule) and maint only through an effect-less toleration
    in.pod_masks(MakePod("p").Toleration("gpu", "Exists", "", kNoSchedule).Toleration("maint", "Exists", "", "")
                     .NodeSelector({{"pool", "gpu"}}).NodeAffinityIn("zone", {"z2", "z1"})
                     .PreferredTerm(50, {{{"zone", "In", {"z1"}}}}).PreferredTerm(0, {{{"x", "Exists", {}}}}).Obj(),
                 &rec);
    CHECK_EQ(rec.tol_hard, (uint64_t)1);
    CHECK_EQ(rec.tol_soft, (uint64_t)2);
    CHECK_EQ(rec.n_req_terms, 1);
    CHECK_EQ(rec.n_pref_terms, 1);  // the weight-0 term is dropped
    CHECK_EQ(rec.pref_weight[0], 50);
    in.label_bits(n, lb);  // requirements interned by the pod: pool In [gpu], zone In [z1 z2], zone In [z1]
    CHECK_EQ(in.n_requirements(), 3);
    CHECK_EQ(lb[0], (uint64_t)7);
    CHECK_EQ((rec.sel[0] & ~lb[0]), (uint64_t)0);
    // a toleration with effect NoSchedule does not tolerate PreferNoSchedule taints for scoring
    qs_pod r2{};
    in.pod_masks(MakePod("q").Toleration("maint", "Exists", "", kNoSchedule).Obj(), &r2);
    CHECK_EQ(r2.tol_soft, (uint64_t)0);
    // an empty required term matches nothing: it carries the reserved never-bit
    qs_pod r3{};
    in.pod_masks(MakePod("e").RequiredTerm(NodeSelectorTerm{}).Obj(), &r3);
    CHECK_EQ(r3.req_terms[0][1], 1ULL << 63);
    // dictionary limits
    Interner full;
    bool threw = false;
    try {
        for (int i = 0; i < 65; ++i) full.taint_bit({"k" + std::to_string(i), "v", kNoSchedule});
    } catch (const DictionaryFull &) { threw = true; }
    CHECK(threw);
    threw = false;
    try {
        qs_pod r4{};
        auto w = MakePod("many");
        for (int i = 0; i < 5; ++i) w.NodeAffinityIn("zone", {"z" + std::to_string(i)});
        in.pod_masks(w.Obj(), &r4);
    } catch (const std::invalid_argument &) { threw = true; }
    CHECK(threw);
}

static void test_pod_resources() {
    // UP component-helpers/resource#PodRequests shapes (spec S2) and ComputePodQOS (S3)
    PodResources r = ComputePodResources(MakePod().Req({{kCPU, "1"}, {kMemory, "1Gi"}}).Req({{kCPU, "500m"}}).Obj());
    CHECK_EQ(r.cpu, (int64_t)1500);
    CHECK_EQ(r.mem, (int64_t)1 << 30);
    CHECK_EQ(r.nz_cpu, (int64_t)1500);
    CHECK_EQ(r.nz_mem, ((int64_t)1 << 30) + 200 * (1 << 20));  // second container: 200Mi default
    CHECK_EQ(r.qos, (int)QS_QOS_BURSTABLE);
    r = ComputePodResources(MakePod().Req({{kCPU, "1"}}).InitReq({{kCPU, "3"}}).Obj());
    CHECK_EQ(r.cpu, (int64_t)3000);  // max(sum, max init)
    r = ComputePodResources(MakePod().Req({{kCPU, "1"}}).SidecarReq({{kCPU, "1"}}).InitReq({{kCPU, "2"}}).Obj());
    CHECK_EQ(r.cpu, (int64_t)3000);  // sidecar adds to the sum (2) and to the later init (1+2=3)
    r = ComputePodResources(MakePod().Req({}).Obj());
    CHECK_EQ(r.cpu, (int64_t)0);
    CHECK_EQ(r.nz_cpu, (int64_t)100);
    CHECK_EQ(r.qos, (int)QS_QOS_BESTEFFORT);
    r = ComputePodResources(MakePod().ReqLim({{kCPU, "2"}, {kMemory, "1Gi"}}, {{kCPU, "2"}, {kMemory, "1Gi"}}).Obj());
    CHECK_EQ(r.qos, (int)QS_QOS_GUARANTEED);
    r = ComputePodResources(MakePod().Req({{kCPU, "1"}}).Overhead({{kCPU, "250m"}, {kMemory, "120Mi"}}).Obj());
    CHECK_EQ(r.cpu, (int64_t)1250);
    CHECK_EQ(r.mem, (int64_t)120 << 20);
    r = ComputePodResources(MakePod().Req({{kCPU, "1"}, {"amd.com/gpu", "2"}}).Obj(), {"amd.com/gpu"});
    CHECK_EQ(r.scalar["amd.com/gpu"], (int64_t)2);
}

static void test_qos_sort_and_fit_error() {
    auto reg = QoSRegistry(nullptr);
    auto qs = std::dynamic_pointer_cast<QueueSortPlugin>(reg[kQoSSort](nullptr));
    QueuedPodInfo g, b, e, b_hi;
    g.res.qos = 2; g.arrival = 3;
    b.res.qos = 1; b.arrival = 1;
    b_hi.res.qos = 1; b_hi.pod.priority = 10; b_hi.arrival = 2;
    e.res.qos = 0; e.arrival = 0;
    CHECK(qs->Less(g, b));
    CHECK(qs->Less(b_hi, b));
    CHECK(qs->Less(b, e));
    CHECK(!qs->Less(e, g));
    CHECK_EQ(FitErrorMessage(3, {{"Insufficient cpu", 2}, {"Too many pods", 1}}),
             std::string("0/3 nodes are available: 1 Too many pods, 2 Insufficient cpu."));
}

// =============================================================================================
// GPU tests
// =============================================================================================
static qs_config default_cfg(bool taint = false, bool affinity = false) {
    qs_config c;
    qs_config_default(&c);
    c.enable_taint = taint;
    c.enable_affinity = affinity;
    return c;
}

// The AMD-GPU cluster configuration: LeastAllocated {cpu:1, memory:1, amd.com/gpu:5},
// BalancedAllocation over [cpu, memory, amd.com/gpu] (amd.com/gpu = extended resource 0).
static qs_config gpu_scoring_cfg(bool taint, bool affinity) {
    qs_config c = default_cfg(taint, affinity);
    c.n_fit_resources = 3;
    c.fit_resources[0] = {QS_RES_CPU, 1};
    c.fit_resources[1] = {QS_RES_MEMORY, 1};
    c.fit_resources[2] = {QS_RES_EXT0, 5};
    c.n_balanced_resources = 3;
    c.balanced_resources[0] = QS_RES_CPU;
    c.balanced_resources[1] = QS_RES_MEMORY;
    c.balanced_resources[2] = QS_RES_EXT0;
    return c;
}

// Scores of one score plugin (weight 1) for `pod` on every node, through PreFilter + Score.
static std::vector<int64_t> plugin_scores(const qs_config &cfg, const std::vector<Node> &nodes,
                                          const Pod &pod, const char *plugin,
                                          std::vector<Code> *filter_codes = nullptr) {
    auto backend = std::make_shared<GpuBackend>(cfg);
    Registry reg = QoSRegistry(backend);
    Profile prof{"test", kQoSSort, {{kQoSGPU}}, {{kQoSGPU}}, {{plugin, 1}}, {{kQoSGPU}}};
    Scheduler sched(reg, {prof}, nullptr);
    for (const auto &n : nodes) sched.AddNode(n);
    Framework fw(prof, reg, &sched);
    CycleState st;
    st.Write(kPodResourcesKey, std::make_shared<PodResourcesState>(ComputePodResources(pod, sched.ExtendedResourceNames())));
    auto [pfr, s] = fw.RunPreFilterPlugins(st, pod);
    CHECK(s.IsSuccess());
    std::vector<const NodeInfo *> all;
    for (const auto &ni : sched.NodeInfos()) {
        all.push_back(&ni);
        if (filter_codes) filter_codes->push_back(fw.RunFilterPlugins(st, pod, ni).code());
    }
    auto [tot, ss] = fw.RunScorePlugins(st, pod, all);
    CHECK(ss.IsSuccess());
    return tot;
}

static void test_gpu_least_allocated() {
    // UP least_allocated_test.go cases, recomputed: score = ((cap - req) * 100 / cap) averaged
    const Pod pod = MakePod().Req({{kCPU, "3000m"}, {kMemory, "5000"}}).Obj();
    const std::vector<Node> nodes = {MakeNode("n1").Capacity({{kCPU, "4000m"}, {kMemory, "10000"}}).Obj(),
                                     MakeNode("n2").Capacity({{kCPU, "6000m"}, {kMemory, "10000"}}).Obj()};
    auto s = plugin_scores(default_cfg(), nodes, pod, kQoSGPULeastAllocated);
    CHECK_EQ(s[0], (int64_t)37);  // ((4000-3000)*100/4000 + (10000-5000)*100/10000) / 2 = (25+50)/2
    CHECK_EQ(s[1], (int64_t)50);  // (50 + 50) / 2
    // nothing requested: non-zero defaults 100m / 200Mi count (useRequested = false)
    const Pod empty = MakePod().Req({}).Obj();
    const std::vector<Node> big = {MakeNode("b").Capacity({{kCPU, "4000m"}, {kMemory, "2000Mi"}}).Obj()};
    s = plugin_scores(default_cfg(), big, empty, kQoSGPULeastAllocated);
    CHECK_EQ(s[0], (int64_t)93);  // cpu 3900*100/4000 = 97, memory 1800Mi*100/2000Mi = 90 -> 187/2
}

static void test_gpu_balanced() {
    // UP balanced_allocation_test.go shape: fractions use Requested (no defaults), truncation
    const Pod pod = MakePod().Req({{kCPU, "3000m"}, {kMemory, "5000"}}).Obj();
    const std::vector<Node> nodes = {MakeNode("n1").Capacity({{kCPU, "4000m"}, {kMemory, "10000"}}).Obj(),
                                     MakeNode("n2").Capacity({{kCPU, "6000m"}, {kMemory, "10000"}}).Obj()};
    auto s = plugin_scores(default_cfg(), nodes, pod, kQoSGPUBalancedAllocation);
    CHECK_EQ(s[0], (int64_t)87);   // |0.75 - 0.5| / 2 = 0.125 -> (1 - 0.125) * 100 = 87.5 -> 87
    CHECK_EQ(s[1], (int64_t)100);  // 0.5 vs 0.5
}

static void test_gpu_fit_filter() {
    // UP fit_test.go shapes: the device rejects, the host explains (FitError reasons)
    auto backend = std::make_shared<GpuBackend>(default_cfg());
    Scheduler sched(QoSRegistry(backend), QoSProfiles(backend->config()), QoSProfileOf);
    sched.AddNode(MakeNode("small").Capacity({{kCPU, "1"}, {kMemory, "1Gi"}, {kPods, "32"}}).Obj());
    sched.AddNode(MakeNode("full").Capacity({{kCPU, "8"}, {kMemory, "8Gi"}, {kPods, "0"}}).Obj());
    sched.AddNode(MakeNode("gpu").Capacity({{kCPU, "8"}, {kMemory, "8Gi"}, {"amd.com/gpu", "1"}}).Obj());
    sched.AddPod(MakePod("big").Req({{kCPU, "2"}, {kMemory, "2Gi"}, {"amd.com/gpu", "2"}}).Obj());
    sched.AddPod(MakePod("fits").Req({{kCPU, "2"}, {kMemory, "2Gi"}}).Obj());
    auto res = sched.Run();
    CHECK_EQ(res.size(), (size_t)2);
    CHECK_EQ(res[0].suggested_host, std::string(""));
    CHECK_EQ(res[0].status.code(), Code::Unschedulable);
    // small: cpu + memory + gpu; full: no pod slot + gpu; gpu: only one device
    CHECK_EQ(res[0].status.Message(), std::string("0/3 nodes are available: 1 Insufficient cpu, 1 Insufficient memory, "
                                                  "1 Too many pods, 3 Insufficient amd.com/gpu."));
    CHECK_EQ(res[1].suggested_host, std::string("gpu"));  // 'full' has no pod slots, 'small' too small
}

static void test_gpu_taint_affinity_scores() {
    // taint_toleration_test.go / node_affinity_test.go shapes with reverse / plain normalization
    const qs_config cfg = default_cfg(true, true);
    const std::vector<Node> nodes = {
        MakeNode("a").Capacity({{kCPU, "8"}, {kMemory, "8Gi"}}).Label("disk", "ssd").Obj(),
        MakeNode("b").Capacity({{kCPU, "8"}, {kMemory, "8Gi"}}).Taint("t1", "x", kPreferNoSchedule).Obj(),
        MakeNode("c").Capacity({{kCPU, "8"}, {kMemory, "8Gi"}}).Taint("t1", "x", kPreferNoSchedule)
            .Taint("t2", "y", kPreferNoSchedule).Label("disk", "ssd").Label("zone", "z1").Obj(),
        MakeNode("d").Capacity({{kCPU, "8"}, {kMemory, "8Gi"}}).Taint("hard", "1", kNoSchedule).Obj()};
    const Pod pod = MakePod().Req({{kCPU, "1"}})
                        .PreferredTerm(30, {{{"disk", "In", {"ssd"}}}})
                        .PreferredTerm(70, {{{"zone", "Exists", {}}}})
                        .Toleration("t2", "Exists", "", kPreferNoSchedule).Obj();
    std::vector<Code> codes;
    auto tt = plugin_scores(cfg, nodes, pod, kQoSGPUTaintToleration, &codes);
    // intolerable PreferNoSchedule counts: a 0, b 1, c 1 (t2 tolerated), d infeasible (hard taint)
    CHECK_EQ(codes[3], Code::UnschedulableAndUnresolvable);
    CHECK_EQ(codes[0], Code::Success);
    CHECK_EQ(tt[0], (int64_t)100);
    CHECK_EQ(tt[1], (int64_t)0);   // 100 - 100*1/1
    CHECK_EQ(tt[2], (int64_t)0);
    auto na = plugin_scores(cfg, nodes, pod, kQoSGPUNodeAffinity);
    // raw: a 30, b 0, c 100 -> normalized by max 100 over feasible nodes
    CHECK_EQ(na[0], (int64_t)30);
    CHECK_EQ(na[1], (int64_t)0);
    CHECK_EQ(na[2], (int64_t)100);
}

// ---- the whole loop on a config-4 cluster built from k8s objects (spec/synth.md G2/G3) --------
static void test_gpu_schedule_one_loop_parity() {
    const uint32_t n = 600, p = 14000;  // ~23 pods per node: the cluster fills up
    const uint64_t seed = 0x5EED0004;
    std::vector<Node> nodes;
    std::vector<Pod> pods;
    synth_objects(4, seed, n, p, &nodes, &pods);
    const qs_config cfg = default_cfg(true, true);
    auto backend = std::make_shared<GpuBackend>(cfg);
    Scheduler sched(QoSRegistry(backend), QoSProfiles(cfg), QoSProfileOf);
    for (const auto &x : nodes) sched.AddNode(x);
    for (const auto &x : pods) sched.AddPod(x);
    const auto res = sched.Run();
    std::vector<int32_t> loop(p, -2);
    for (const auto &r : res) loop[r.arrival] = r.node_index;

    // the same cluster through the generator's fixed bit assignment: stream path and oracle
    std::vector<int64_t> col[10];
    for (auto &v : col) v.assign(n, 0);
    std::vector<int64_t> ae(2 * n), re(2 * n);
    std::vector<uint64_t> th(n), ts(n), lb(2 * n);
    qs_node_soa_out out{col[0].data(), col[1].data(), ae.data(), col[2].data(), col[3].data(), col[4].data(),
                        re.data(), col[5].data(), col[6].data(), col[7].data(), th.data(), ts.data(), lb.data(), nullptr};
    std::vector<qs_pod> recs(p);
    CHECK_EQ((int)qs_synth_generate(4, seed, n, p, &out, recs.data()), (int)QS_OK);
    qs_ctx *ctx = nullptr;
    CHECK_EQ((int)qs_open(&cfg, 0, &ctx), (int)QS_OK);
    qs_node_soa in{col[0].data(), col[1].data(), ae.data(), col[2].data(), col[3].data(), col[4].data(),
                   re.data(), col[5].data(), col[6].data(), col[7].data(), th.data(), ts.data(), lb.data(), nullptr};
    CHECK_EQ((int)qs_nodes_load(ctx, &in, n), (int)QS_OK);
    std::vector<int32_t> stream(p);
    qs_stats stats;
    CHECK_EQ((int)qs_schedule_stream(ctx, recs.data(), p, QS_MODE_EXACT, stream.data(), &stats), (int)QS_OK);
    qs_close(ctx);

    // oracle (test infrastructure) on the generator's arrays
    std::vector<int64_t> o[10];
    for (auto &v : o) v.assign(n, 0);
    std::vector<int64_t> oae(2 * n), ore(2 * n);
    std::vector<uint64_t> oth(n), ots(n), olb(2 * n);
    or_nodes on{n, o[0].data(), o[1].data(), oae.data(), o[2].data(), o[3].data(), o[4].data(), ore.data(),
                o[5].data(), o[6].data(), o[7].data(), oth.data(), ots.data(), olb.data(), nullptr};
    std::vector<int64_t> prc(p), prm(p), pre(2 * p), pzc(p), pzm(p);
    std::vector<int32_t> pq(p), ppr(p), pnr(p), pnp(p), ppw(4 * p);
    std::vector<uint64_t> pth(p), pts(p), psel(2 * p), prt(8 * p), ppt(8 * p);
    or_pods op{p, prc.data(), prm.data(), pre.data(), pzc.data(), pzm.data(), pq.data(), ppr.data(), pth.data(),
               pts.data(), psel.data(), pnr.data(), pnp.data(), prt.data(), ppt.data(), ppw.data(), nullptr, nullptr};
    or_generate(4, seed, &on, &op);
    const or_config oc = oracle_cfg(cfg);
    std::vector<int32_t> oracle(p);
    or_schedule(&oc, &on, &op, oracle.data(), nullptr, nullptr, 8);

    int diff_stream = 0, diff_oracle = 0, unsched = 0;
    for (uint32_t j = 0; j < p; ++j) {
        diff_stream += loop[j] != stream[j];
        diff_oracle += loop[j] != oracle[j];
        unsched += loop[j] < 0;
    }
    std::printf("  ScheduleOne loop: %u pods on %u nodes, %d unschedulable, %d differ from qs_schedule_stream, "
                "%d from the oracle; %llu full table loads, %llu row upserts\n",
                p, n, unsched, diff_stream, diff_oracle, (unsigned long long)backend->full_loads(),
                (unsigned long long)backend->row_upserts());
    CHECK_EQ(diff_stream, 0);
    CHECK_EQ(diff_oracle, 0);
    CHECK(unsched > 0 && unsched < (int)p);
}

// Parallelizer::Until: an exception thrown by a piece of work on any thread reaches the caller once
// every worker has left the work function, and the pool stays usable.
static void test_parallelizer_exceptions() {
    Parallelizer par(8);
    for (int rep = 0; rep < 20; ++rep) {
        std::atomic<int> ran{0};
        bool thrown = false;
        try {
            par.Until(1000, [&](int i) {
                ran.fetch_add(1);
                if (i == 37 + rep) throw std::runtime_error("piece failed");
            });
        } catch (const std::runtime_error &e) {
            thrown = std::string(e.what()) == "piece failed";
        }
        CHECK(thrown);
        CHECK(ran.load() <= 1000);
        std::atomic<int> sum{0};
        par.Until(1000, [&](int i) { sum.fetch_add(i); });
        CHECK_EQ(sum.load(), 999 * 1000 / 2);
    }
}

// ---- the CPU reference plugins (host/cpu_plugins.cpp) ------------------------------------------
// One pod on one node through the CPU plugins' Filter / Score, against the oracle's scorers.
static void test_cpu_plugin_scores() {
    qs_config cfg = default_cfg(true, true);
    struct Tc {
        const char *cpu, *mem, *rcpu, *rmem;
    } tcs[] = {{"4000m", "8Gi", "1000m", "2Gi"}, {"16", "64Gi", "3500m", "7Gi"}, {"2", "1Gi", "100m", "2Gi"}};
    for (const auto &tc : tcs) {
        Scheduler sched(CPURegistry(cfg), CPUProfiles(cfg), CPUProfileOf, 1);
        sched.AddNode(MakeNode("n0").Capacity({{kCPU, tc.cpu}, {kMemory, tc.mem}, {kPods, "110"}}).Obj());
        Pod pod = MakePod("p").ReqLim({{kCPU, tc.rcpu}, {kMemory, tc.rmem}}, {}).Obj();
        auto reg = CPURegistry(cfg);
        auto fit = std::dynamic_pointer_cast<ScorePlugin>(reg[kNodeResourcesFit](&sched));
        auto bal = std::dynamic_pointer_cast<ScorePlugin>(reg[kNodeResourcesBalancedAllocation](&sched));
        auto flt = std::dynamic_pointer_cast<FilterPlugin>(reg[kNodeResourcesFit](&sched));
        CycleState st;
        const PodResources r = ComputePodResources(pod);
        const NodeInfo &ni = sched.NodeInfos()[0];
        const int64_t la = fit->Score(st, pod, "n0").first, ba = bal->Score(st, pod, "n0").first;
        CHECK_EQ(la, or_least_allocated(ni.allocatable.milli_cpu, r.nz_cpu, ni.allocatable.memory, r.nz_mem, 1, 1));
        CHECK_EQ(ba, or_balanced(ni.allocatable.milli_cpu, r.cpu, ni.allocatable.memory, r.mem));
        const bool fits = r.cpu <= ni.allocatable.milli_cpu && r.mem <= ni.allocatable.memory;
        const Status fs = flt->Filter(st, pod, ni);
        CHECK_EQ(fs.IsSuccess(), fits);
        if (!fits) CHECK(fs.Message().find("Insufficient memory") != std::string::npos);
    }
}

// spec/kat.md K10 / K11 / K12 (configurable scoring resources) through the CPU plugins' Score.
static void test_cpu_plugin_scores_resource_lists() {
    const qs_config cfg = gpu_scoring_cfg(false, false);
    struct Tc {
        const char *node_cpu, *node_mem, *node_gpu, *used_cpu, *used_mem, *used_gpu, *cpu, *mem, *gpu;
        int64_t la, ba;
    } tcs[] = {
        // K10 / K11: used (2000m, 8Gi, 2) + pod (2000m, 8Gi, 4) on (8000m, 32Gi, 8)
        {"8000m", "32Gi", "8", "2000m", "8Gi", "2", "2000m", "8Gi", "4", 32, 88},
        // K10b: the pod requests no gpu -> gpu skipped in both lists
        {"8000m", "32Gi", "8", "2000m", "8Gi", "2", "2000m", "8Gi", nullptr, 50, 100},
        // K12: three resources at 4/5 -> float64 std > 0 -> 99 (exact arithmetic: 100)
        {"4000m", "10Gi", "5", nullptr, nullptr, nullptr, "3200m", "8Gi", "4", 20, 99},
    };
    for (const auto &tc : tcs) {
        Scheduler sched(CPURegistry(cfg), CPUProfiles(cfg), CPUProfileOf, 1);
        sched.AddNode(MakeNode("n0").Capacity({{kCPU, tc.node_cpu}, {kMemory, tc.node_mem}, {"amd.com/gpu", tc.node_gpu},
                                               {kPods, "110"}}).Obj());
        if (tc.used_cpu) {  // the node's usage: one pod scheduled (and assumed) there first
            sched.AddPod(MakePod("used").ReqLim({{kCPU, tc.used_cpu}, {kMemory, tc.used_mem}, {"amd.com/gpu", tc.used_gpu}}, {}).Obj());
            const auto placed = sched.Run();
            CHECK(placed.size() == 1 && placed[0].node_index == 0);
        }
        ResourceList req{{kCPU, tc.cpu}, {kMemory, tc.mem}};
        if (tc.gpu) req["amd.com/gpu"] = tc.gpu;
        Pod pod = MakePod("p").ReqLim(req, {}).Obj();
        auto reg = CPURegistry(cfg);
        auto fit = std::dynamic_pointer_cast<ScorePlugin>(reg[kNodeResourcesFit](&sched));
        auto bal = std::dynamic_pointer_cast<ScorePlugin>(reg[kNodeResourcesBalancedAllocation](&sched));
        CycleState st;
        CHECK_EQ(fit->Score(st, pod, "n0").first, tc.la);
        CHECK_EQ(bal->Score(st, pod, "n0").first, tc.ba);
    }
}

// The whole ScheduleOne loop with the CPU plugins (16-worker Parallelizer for config 2, 4 for config
// 4) on spec/synth.md clusters built as k8s objects, pod by pod against the oracle.
static void cpu_loop_parity(int config, uint32_t n, uint32_t p, int workers, const qs_config *over = nullptr) {
    const uint64_t seed = 0x5EED0000ull + (uint64_t)config;
    std::vector<Node> nodes;
    std::vector<Pod> pods;
    synth_objects(config, seed, n, p, &nodes, &pods);
    const qs_config cfg = over ? *over : default_cfg(config == 4, config == 4);
    Scheduler sched(CPURegistry(cfg), CPUProfiles(cfg), CPUProfileOf, workers);
    for (const auto &x : nodes) sched.AddNode(x);
    for (const auto &x : pods) sched.AddPod(x);
    const auto res = sched.Run();
    std::vector<int32_t> loop(p, -2);
    for (const auto &r : res) loop[r.arrival] = r.node_index;
    std::vector<int64_t> o[10];
    for (auto &v : o) v.assign(n, 0);
    std::vector<int64_t> oae(2 * n), ore(2 * n);
    std::vector<uint64_t> oth(n), ots(n), olb(2 * n);
    or_nodes on{n, o[0].data(), o[1].data(), oae.data(), o[2].data(), o[3].data(), o[4].data(), ore.data(),
                o[5].data(), o[6].data(), o[7].data(), oth.data(), ots.data(), olb.data(), nullptr};
    std::vector<int64_t> prc(p), prm(p), pre(2 * p), pzc(p), pzm(p);
    std::vector<int32_t> pq(p), ppr(p), pnr(p), pnp(p), ppw(4 * p);
    std::vector<uint64_t> pth(p), pts(p), psel(2 * p), prt(8 * p), ppt(8 * p);
    or_pods op{p, prc.data(), prm.data(), pre.data(), pzc.data(), pzm.data(), pq.data(), ppr.data(), pth.data(),
               pts.data(), psel.data(), pnr.data(), pnp.data(), prt.data(), ppt.data(), ppw.data(), nullptr, nullptr};
    or_generate(config, seed, &on, &op);
    const or_config oc = oracle_cfg(cfg);
    std::vector<int32_t> oracle(p);
    or_schedule(&oc, &on, &op, oracle.data(), nullptr, nullptr, 4);
    int diff = 0, unsched = 0;
    for (uint32_t j = 0; j < p; ++j) {
        diff += loop[j] != oracle[j];
        unsched += loop[j] < 0;
    }
    std::printf("  CPU plugins, config %d%s: %u pods on %u nodes (%d workers), %d unschedulable, %d differ from the oracle\n",
                config, cfg.n_fit_resources ? " (gpu scoring resources)" : "", p, n, workers, unsched, diff);
    CHECK_EQ(diff, 0);
    if (config == 4) CHECK(unsched > 0 && unsched < (int)p);
}
static void test_cpu_loop_config1() { cpu_loop_parity(1, 100, 1000, 16); }  // BASELINE configs[0] at its size
static void test_cpu_loop_config2() { cpu_loop_parity(2, 300, 9000, 16); }
static void test_cpu_loop_config4() { cpu_loop_parity(4, 400, 9000, 4); }
static void test_cpu_loop_config4_gpu_scoring() {
    const qs_config c = gpu_scoring_cfg(true, true);
    cpu_loop_parity(4, 400, 6000, 4, &c);
}

int main(int argc, char **argv) {
    const bool gpu = argc > 1 && std::strcmp(argv[1], "--gpu") == 0;
    std::vector<Case> cases;
    if (!gpu) {
        cases = {{"quantity", test_quantity}, {"tolerations", test_tolerations},
                 {"requirements", test_requirements}, {"interner", test_interner},
                 {"pod_resources", test_pod_resources}, {"qos_sort_fit_error", test_qos_sort_and_fit_error},
                 {"parallelizer_exceptions", test_parallelizer_exceptions},
                 {"cpu_plugin_scores", test_cpu_plugin_scores},
                 {"cpu_plugin_scores_resource_lists", test_cpu_plugin_scores_resource_lists},
                 {"cpu_loop_config1", test_cpu_loop_config1}, {"cpu_loop_config2", test_cpu_loop_config2},
                 {"cpu_loop_config4", test_cpu_loop_config4},
                 {"cpu_loop_config4_gpu_scoring", test_cpu_loop_config4_gpu_scoring}};
    } else {
        cases = {{"gpu_least_allocated", test_gpu_least_allocated}, {"gpu_balanced", test_gpu_balanced},
                 {"gpu_fit_filter", test_gpu_fit_filter}, {"gpu_taint_affinity_scores", test_gpu_taint_affinity_scores},
                 {"gpu_schedule_one_loop_parity", test_gpu_schedule_one_loop_parity}};
    }
    for (const auto &c : cases) {
        const int before = g_fail;
        try {
            c.fn();
        } catch (const std::exception &e) {
            ++g_fail;
            std::fprintf(stderr, "  FAIL %s: exception: %s\n", c.name, e.what());
        }
        std::printf("%s %s\n", g_fail == before ? "PASS" : "FAIL", c.name);
    }
    std::printf("%d checks, %d failures\n", g_checks, g_fail);
    return g_fail ? 1 : 0;
}
