"""scheduler_perf-style workload files -> node table and pod stream.

A workload file is the subset of upstream's scheduler_perf test-case format
(UP test/integration/scheduler_perf/config/performance-config.yaml, op codes of
UP test/integration/scheduler_perf/scheduler_perf.go) that describes the cluster and the pod
stream the hot path schedules:

    - name: TestCase
      workloadTemplate:
      - opcode: createNodes
        countParam: $initNodes            # or count: 500
        nodeTemplate: {metadata: {labels}, spec: {taints}, status: {allocatable}}
        labelStrategy: {key: topology.kubernetes.io/zone, values: [z0, z1, z2]}   # optional
      - opcode: createPods
        countParam: $measurePods
        podTemplate: {spec: {containers, initContainers, overhead, priority, nodeSelector,
                             tolerations, affinity: {nodeAffinity}}}
      workloads:
      - name: 500Nodes
        params: {initNodes: 500, measurePods: 1000}

(upstream reads the templates from nodeTemplatePath / podTemplatePath files; here they are inline,
and `labelStrategy` plays the part of upstream's labelNodePrepareStrategy: node i gets
values[i % len(values)]).  `load(path, workload)` returns the canonical node columns and pod
records of include/qsched.h, built with the same semantics as the C++ framework layer
(custom-k8s-scheduler_amd/host/k8s.cpp quantities, host/intern.cpp taint / requirement
dictionaries) and spec/semantics.md S1–S3.  Parsing is host-side test/bench plumbing; the product
path is the C ABI it feeds.
"""
from fractions import Fraction
import re

import numpy as np
import yaml

from . import POD_DTYPE, QS_MAX_EXT, QS_MAX_TERMS, empty_nodes, pod_from_containers

_SUFFIX = {"": 1, "m": Fraction(1, 1000), "k": 10**3, "M": 10**6, "G": 10**9, "T": 10**12,
           "P": 10**15, "E": 10**18, "Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40,
           "Pi": 2**50, "Ei": 2**60}
_QTY = re.compile(r"^([+-]?[0-9]*\.?[0-9]*)(?:([eE][+-]?[0-9]+)|(Ki|Mi|Gi|Ti|Pi|Ei|[mkMGTPE]))?$")
_HARD = ("NoSchedule", "NoExecute")
_NEVER_BIT = 127  # reserved requirement bit no node carries (empty selector terms)


def parse_quantity(q) -> Fraction:
    """resource.Quantity (UP apimachinery/pkg/api/resource#ParseQuantity) as an exact rational."""
    if isinstance(q, (int, float)) and not isinstance(q, bool):
        return Fraction(str(q))
    m = _QTY.match(str(q).strip())
    if not m or m.group(1) in ("", "+", "-", "."):
        raise ValueError(f"invalid quantity {q!r}")
    v = Fraction(m.group(1))
    if m.group(2):
        return v * Fraction(10) ** int(m.group(2)[1:])
    return v * _SUFFIX[m.group(3) or ""]


def _ceil(x: Fraction) -> int:
    return -((-x.numerator) // x.denominator)


def milli_value(q) -> int:  # Quantity.MilliValue(): rounds up
    return _ceil(parse_quantity(q) * 1000)


def value(q) -> int:  # Quantity.Value(): rounds up
    return _ceil(parse_quantity(q))


def tolerates(tol, taint) -> bool:
    """UP core/v1/toleration.go#ToleratesTaint."""
    if tol.get("effect") and tol["effect"] != taint.get("effect"):
        return False
    if tol.get("key") and tol["key"] != taint.get("key"):
        return False
    op = tol.get("operator") or "Equal"
    if op == "Equal":
        return (tol.get("value") or "") == (taint.get("value") or "")
    return op == "Exists"


def requirement_matches(req, labels) -> bool:
    """UP labels.Requirement.Matches for node-selector operators (invalid selectors match none)."""
    key, op, vals = req
    has = key in labels
    if op in ("In", "NotIn"):
        if not vals:
            return False
        inn = has and labels[key] in vals
        return inn if op == "In" else not inn
    if op == "Exists":
        return not vals and has
    if op == "DoesNotExist":
        return not vals and not has
    if op in ("Gt", "Lt"):
        try:
            want, got = int(vals[0]), int(labels[key]) if has else None
        except (ValueError, IndexError):
            return False
        if len(vals) != 1 or got is None:
            return False
        return got > want if op == "Gt" else got < want
    return False


class Interner:
    """Taint (64) and node-selector requirement (127 + never) dictionaries, as host/intern.cpp."""

    def __init__(self):
        self.taints, self._tix = [], {}
        self.reqs, self._rix = [], {}
        self.ext, self._eix = [], {}

    def taint_bit(self, t) -> int:
        k = (t.get("key", ""), t.get("value", "") or "", t.get("effect", ""))
        if k not in self._tix:
            if len(self.taints) >= 64:
                raise ValueError("more than 64 distinct taints (key, value, effect) in the cluster")
            self._tix[k] = len(self.taints)
            self.taints.append({"key": k[0], "value": k[1], "effect": k[2]})
        return self._tix[k]

    def requirement_bit(self, key, op, vals) -> int:
        vals = tuple(sorted(vals)) if op in ("In", "NotIn") else tuple(vals)
        k = (key, op, vals)
        if k not in self._rix:
            if len(self.reqs) >= _NEVER_BIT:
                raise ValueError("more than 127 distinct node-selector requirements in the pod stream")
            self._rix[k] = len(self.reqs)
            self.reqs.append(k)
        return self._rix[k]

    def ext_slot(self, name) -> int:
        if name not in self._eix:
            if len(self.ext) >= QS_MAX_EXT:
                raise ValueError(f"more than {QS_MAX_EXT} extended resources")
            self._eix[name] = len(self.ext)
            self.ext.append(name)
        return self._eix[name]

    def term_mask(self, term):
        m = [0, 0]
        exprs = (term or {}).get("matchExpressions") or []
        bits = [_NEVER_BIT] if not exprs else [
            self.requirement_bit(e["key"], e["operator"], list(e.get("values") or [])) for e in exprs]
        for b in bits:
            m[b >> 6] |= 1 << (b & 63)
        return m

    def label_bits(self, labels):
        m = [0, 0]
        for b, r in enumerate(self.reqs):
            if requirement_matches(r, labels):
                m[b >> 6] |= 1 << (b & 63)
        return m


_STD = ("cpu", "memory", "pods", "ephemeral-storage")


def _is_ext(name) -> bool:  # extended resources: domain-prefixed names (amd.com/gpu, ...)
    return name not in _STD and "/" in name


def _count(op, params):
    if "count" in op:
        return int(op["count"])
    p = str(op["countParam"]).lstrip("$")
    return int(params[p])


def load(path_or_text, workload=None, testcase=None, names=False):
    """Parse a workload file; returns (nodes, pods, profile) for the chosen test case/workload.

    nodes: canonical node columns (qsched.empty_nodes layout); pods: POD_DTYPE array in creation
    order; profile: {"enable_taint", "enable_affinity"} switched on when the file uses taints,
    tolerations, node selectors or node affinity.  names=True adds a fourth item, {"taints":
    {bit: "key: value"}}, the interned taint dictionary FitError texts name taints with
    (qsched.fit_error_message's taint_names)."""
    text = path_or_text
    if "\n" not in str(path_or_text):
        with open(path_or_text) as f:
            text = f.read()
    cases = yaml.safe_load(text)
    if isinstance(cases, dict):
        cases = [cases]
    case = next((c for c in cases if testcase in (None, c.get("name"))), None)
    if case is None:
        raise KeyError(f"test case {testcase!r} not found")
    wls = case.get("workloads") or [{"name": "default", "params": {}}]
    wl = next((w for w in wls if workload in (None, w.get("name"))), None)
    if wl is None:
        raise KeyError(f"workload {workload!r} not found")
    params = wl.get("params") or {}
    node_specs, pod_specs = [], []
    for op in case["workloadTemplate"]:
        code = op["opcode"]
        if code == "createNodes":
            tmpl = op.get("nodeTemplate") or {}
            strat = op.get("labelStrategy")
            for i in range(_count(op, params)):
                labels = dict((tmpl.get("metadata") or {}).get("labels") or {})
                if strat:
                    labels[strat["key"]] = strat["values"][len(node_specs) % len(strat["values"])]
                node_specs.append((tmpl, labels))
        elif code == "createPods":
            tmpl = op.get("podTemplate") or {}
            pod_specs.extend([tmpl] * _count(op, params))
        elif code in ("barrier", "sleep", "startCollectingMetrics", "stopCollectingMetrics"):
            continue
        else:
            raise ValueError(f"unsupported opcode {code!r}")
    it = Interner()
    uses_taint = uses_aff = False
    # nodes: resources and taints (taint dictionary complete before any toleration is evaluated)
    n = len(node_specs)
    nodes = empty_nodes(n)
    for i, (tmpl, _) in enumerate(node_specs):
        alloc = (tmpl.get("status") or {}).get("allocatable") or {}
        nodes["alloc_cpu"][i] = milli_value(alloc.get("cpu", 0))
        nodes["alloc_mem"][i] = value(alloc.get("memory", 0))
        nodes["max_pods"][i] = value(alloc.get("pods", 110))
        for name, q in alloc.items():
            if _is_ext(name):
                nodes["alloc_ext"][i, it.ext_slot(name)] = value(q)
        th = ts = 0
        for t in (tmpl.get("spec") or {}).get("taints") or []:
            uses_taint = True
            b = it.taint_bit(t)
            if t.get("effect") in _HARD:
                th |= 1 << b
            elif t.get("effect") == "PreferNoSchedule":
                ts |= 1 << b
        nodes["taint_hard"][i], nodes["taint_soft"][i] = th, ts
    # pods: S2/S3 through the library, then the interned masks
    pods = np.zeros(len(pod_specs), POD_DTYPE)
    cache = {}
    for j, tmpl in enumerate(pod_specs):
        key = id(tmpl)
        if key not in cache:
            cache[key] = _pod_record(tmpl, it)
        rec, ut, ua = cache[key]
        uses_taint |= ut
        uses_aff |= ua
        pods[j] = rec
    for i, (_, labels) in enumerate(node_specs):
        nodes["label_bits"][i] = it.label_bits(labels)
    prof = {"enable_taint": int(uses_taint), "enable_affinity": int(uses_aff)}
    if names:
        return nodes, pods, prof, {"taints": {b: f"{t['key']}: {t['value']}" for b, t in enumerate(it.taints)}}
    return nodes, pods, prof


def _containers(spec, it):
    out = []
    for kind, lst in (("init", spec.get("initContainers")), ("regular", spec.get("containers"))):
        for c in lst or []:
            res = c.get("resources") or {}
            req, lim = res.get("requests") or {}, res.get("limits") or {}
            d = {"kind": "sidecar" if kind == "init" and c.get("restartPolicy") == "Always" else kind}
            if "cpu" in req:
                d["req_cpu"] = milli_value(req["cpu"])
            if "memory" in req:
                d["req_mem"] = value(req["memory"])
            if "cpu" in lim:
                d["lim_cpu"] = milli_value(lim["cpu"])
            if "memory" in lim:
                d["lim_mem"] = value(lim["memory"])
            ext = [0] * QS_MAX_EXT
            for name, q in req.items():
                if _is_ext(name):
                    ext[it.ext_slot(name)] = value(q)
            for name, q in lim.items():  # extended resources: limits imply equal requests
                if _is_ext(name) and name not in req:
                    ext[it.ext_slot(name)] = value(q)
            d["req_ext"] = ext
            out.append(d)
    return out


def _pod_record(tmpl, it):
    spec = tmpl.get("spec") or {}
    ov = spec.get("overhead")
    overhead = None if not ov else (milli_value(ov.get("cpu", 0)), value(ov.get("memory", 0)))
    rec = pod_from_containers(_containers(spec, it), overhead)
    rec["priority"] = int(spec.get("priority") or 0)
    uses_taint = bool(spec.get("tolerations"))
    th = ts = 0
    for b, t in enumerate(it.taints):
        for tol in spec.get("tolerations") or []:
            if not tolerates(tol, t):
                continue
            if t["effect"] in _HARD:
                th |= 1 << b
            if t["effect"] == "PreferNoSchedule" and (tol.get("effect") or "") in ("", "PreferNoSchedule"):
                ts |= 1 << b
    rec["tol_hard"], rec["tol_soft"] = th, ts
    sel = [0, 0]
    for k, v in (spec.get("nodeSelector") or {}).items():
        b = it.requirement_bit(k, "In", [v])
        sel[b >> 6] |= 1 << (b & 63)
    rec["sel"] = sel
    na = (spec.get("affinity") or {}).get("nodeAffinity") or {}
    req = ((na.get("requiredDuringSchedulingIgnoredDuringExecution") or {}).get("nodeSelectorTerms")) or []
    pref = [p for p in (na.get("preferredDuringSchedulingIgnoredDuringExecution") or []) if p.get("weight", 0)]
    if len(req) > QS_MAX_TERMS or len(pref) > QS_MAX_TERMS:
        raise ValueError(f"more than {QS_MAX_TERMS} node-affinity terms")
    for p in pref:
        if not 0 <= int(p["weight"]) <= 100:
            raise ValueError("preferred term weight outside 0..100")
    rec["n_req_terms"] = len(req)
    for t, term in enumerate(req):
        rec["req_terms"][t] = it.term_mask(term)
    rec["n_pref_terms"] = len(pref)
    for t, p in enumerate(pref):
        rec["pref_terms"][t] = it.term_mask(p.get("preference"))
        rec["pref_weight"][t] = int(p["weight"])
    uses_aff = bool(spec.get("nodeSelector") or req or pref)
    return rec, uses_taint, uses_aff
