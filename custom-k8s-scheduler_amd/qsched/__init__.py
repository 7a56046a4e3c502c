"""qsched — Python binding of libqsched.so (the gfx950 scheduling core behind include/qsched.h).

This is plumbing for tests and ``bench.py``; the product is the C ABI.  Every call goes through
the HIP library: if ``libqsched.so`` is missing, importing the binding succeeds but the first call
raises ``QschedLibraryMissing`` — there is no CPU fallback.

Data model (the same field names as include/qsched.h):
  * nodes: dict of numpy arrays (``alloc_cpu``, ``alloc_mem``, ``alloc_ext`` [n,2], ``max_pods``,
    ``req_cpu``, ``req_mem``, ``req_ext`` [n,2], ``nz_cpu``, ``nz_mem``, ``pods`` int64;
    ``taint_hard``, ``taint_soft`` uint64; ``label_bits`` [n,2] uint64);
  * pods: numpy structured array of ``POD_DTYPE`` (one ``qs_pod`` per element) or the equivalent
    dict of arrays (converted with ``pods_to_struct``).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._abi import (ENGINES, ENGINE_NAMES, EXPORTED, LIB_PATH, POD_DTYPE, QS_ABI_VERSION,
                   QS_MAX_EXT, QS_MAX_SCORE_RES, QS_MAX_TERMS, QS_MODE_BATCHED, QS_MODE_EXACT, QS_OK,
                   RESOURCES, FIT_REASONS, QS_FIT_TAINT, QschedError,
                   QschedLibraryMissing, QsConfig, QsContainer, QsNodeRow, QsNodeSoa, QsStats,
                   load)

__all__ = ["Scheduler", "Config", "POD_DTYPE", "pods_to_struct", "pods_from_struct", "fit_error_message",
           "synth_generate", "dist_unique_id", "empty_nodes", "pod_from_containers", "compute_qos", "load",
           "QschedError", "QschedLibraryMissing", "ENGINES", "EXPORTED", "LIB_PATH"]

MODES = {"exact": QS_MODE_EXACT, "batched": QS_MODE_BATCHED}
NODE_I64 = ["alloc_cpu", "alloc_mem", "max_pods", "req_cpu", "req_mem", "nz_cpu", "nz_mem", "pods"]


def _check(lib, ctx, st):
    if st != QS_OK:
        msg = lib.qs_last_error(ctx).decode() if ctx else ""
        raise QschedError(st, msg)


def _ptr(a):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays passed to the C ABI must be C-contiguous"
    return a.ctypes.data


def empty_nodes(n: int):
    d = {f: np.zeros(n, np.int64) for f in NODE_I64}
    d["alloc_ext"] = np.zeros((n, QS_MAX_EXT), np.int64)
    d["req_ext"] = np.zeros((n, QS_MAX_EXT), np.int64)
    d["taint_hard"] = np.zeros(n, np.uint64)
    d["taint_soft"] = np.zeros(n, np.uint64)
    d["label_bits"] = np.zeros((n, 2), np.uint64)
    d["zone"] = np.zeros(n, np.int32)
    return d


def _soa(nodes, lib_out=False):
    s = QsNodeSoa()
    for f, _ in QsNodeSoa._fields_:
        a = nodes.get(f)
        if a is not None:
            want = (np.uint64 if f in ("taint_hard", "taint_soft", "label_bits") else
                    np.int32 if f == "zone" else np.int64)
            if a.dtype != want or not a.flags["C_CONTIGUOUS"]:
                if lib_out:
                    raise TypeError(f"output column {f} must be C-contiguous {want}")
                a = np.ascontiguousarray(a, dtype=want)
                nodes = dict(nodes)
                nodes[f] = a
        setattr(s, f, _ptr(a))
    return s, nodes  # keep the converted arrays alive with the struct


def pods_to_struct(pods) -> np.ndarray:
    """dict-of-arrays (oracle layout) or structured array -> contiguous POD_DTYPE array."""
    if isinstance(pods, np.ndarray) and pods.dtype == POD_DTYPE:
        return np.ascontiguousarray(pods)
    p = len(pods["req_cpu"])
    out = np.zeros(p, POD_DTYPE)
    for f in POD_DTYPE.names:
        if f in pods:
            out[f] = pods[f]
    return out


def pods_from_struct(arr: np.ndarray):
    return {f: np.ascontiguousarray(arr[f]) for f in POD_DTYPE.names}


class Config(dict):
    """qs_config as a dict; unspecified fields take qs_config_default()."""

    def to_c(self) -> QsConfig:
        lib = load()
        c = QsConfig()
        lib.qs_config_default(ctypes.byref(c))
        for k, v in self.items():
            if k == "engine" and isinstance(v, str):
                v = ENGINES[v]
            if k in ("w_fit", "w_bal"):
                for i in range(3):
                    getattr(c, k)[i] = int(v[i])
            elif k == "fit_resources":  # [(name | id, weight), ...] (spec S5 "Scoring resources")
                v = list(v or [])
                if len(v) > QS_MAX_SCORE_RES:
                    raise ValueError("at most 4 scoring resources")
                c.n_fit_resources = len(v)
                for i, (name, w) in enumerate(v):
                    c.fit_resources[i][0] = RESOURCES[name] if isinstance(name, str) else int(name)
                    c.fit_resources[i][1] = int(w)
            elif k == "balanced_resources":  # [name | id, ...]
                v = list(v or [])
                if len(v) > QS_MAX_SCORE_RES:
                    raise ValueError("at most 4 balanced resources")
                c.n_balanced_resources = len(v)
                for i, name in enumerate(v):
                    c.balanced_resources[i] = RESOURCES[name] if isinstance(name, str) else int(name)
            else:
                setattr(c, k, int(v))
        return c


class Scheduler:
    """One device context (``qs_ctx``) on one GPU."""

    def __init__(self, config=None, device: int = 0, shard=None):
        """shard = (rank, world, unique_id bytes) opens a node-sharded context (qs_open_shard):
        every rank loads the same full table and pod stream; RCCL exchanges the per-window lists.
        unique_id None: the peer-memory mailbox transport (mailbox_export / mailbox_connect)."""
        self.lib = load()
        self.cfg = Config(config or {}).to_c()
        ctx = ctypes.c_void_p()
        if shard is None:
            st = self.lib.qs_open(ctypes.byref(self.cfg), device, ctypes.byref(ctx))
        else:
            rank, world, uid = shard
            buf = None if uid is None else (ctypes.c_uint8 * 128).from_buffer_copy(bytes(uid))
            st = self.lib.qs_open_shard(ctypes.byref(self.cfg), device, rank, world, buf,
                                        ctypes.byref(ctx))
        if st != QS_OK:
            why = self.lib.qs_last_error(None)
            raise QschedError(st, "qs_open failed: " + (why.decode() if why else "no HIP device?"))
        self.ctx = ctx
        self.n = 0

    def mailbox_export(self) -> bytes:
        """qs_dist_mailbox_export: this rank's 64-byte mailbox IPC handle (sharded contexts opened
        without an RCCL id)."""
        buf = (ctypes.c_uint8 * 64)()
        self._chk(self.lib.qs_dist_mailbox_export(self.ctx, buf))
        return bytes(buf)

    def mailbox_connect(self, handles):
        """qs_dist_mailbox_connect with every rank's handle, in rank order."""
        blob = b"".join(bytes(h) for h in handles)
        buf = (ctypes.c_uint8 * len(blob)).from_buffer_copy(blob)
        self._chk(self.lib.qs_dist_mailbox_connect(self.ctx, buf))

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.qs_close(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, st):
        _check(self.lib, self.ctx, st)

    # ---- node table ----
    def load_nodes(self, nodes):
        s, keep = _soa(nodes)
        n = len(nodes["alloc_cpu"])
        self._chk(self.lib.qs_nodes_load(self.ctx, ctypes.byref(s), n))
        self.n = n
        del keep

    def read_nodes(self):
        out = empty_nodes(self.n)
        s, _ = _soa(out, lib_out=True)
        self._chk(self.lib.qs_nodes_read(self.ctx, ctypes.byref(s), self.n))
        return out

    def upsert(self, idx, row: dict, generation=0):
        r = QsNodeRow()
        for f, t in QsNodeRow._fields_:
            if f in row:
                v = row[f]
                if f in ("alloc_ext", "req_ext", "label_bits"):
                    for i, x in enumerate(v):
                        getattr(r, f)[i] = int(x)
                else:
                    setattr(r, f, int(v))
        self._chk(self.lib.qs_node_upsert(self.ctx, idx, ctypes.byref(r), generation))
        if idx == self.n:
            self.n += 1

    def save_table(self):
        self._chk(self.lib.qs_table_save(self.ctx))

    def restore_table(self):
        self._chk(self.lib.qs_table_restore(self.ctx))

    def reserve(self, node, pod):
        p = pods_to_struct(pod) if not isinstance(pod, np.void) else np.array([pod], POD_DTYPE)
        self._chk(self.lib.qs_reserve(self.ctx, node, _ptr(p)))

    def unreserve(self, node, pod):
        p = pods_to_struct(pod) if not isinstance(pod, np.void) else np.array([pod], POD_DTYPE)
        self._chk(self.lib.qs_unreserve(self.ctx, node, _ptr(p)))

    # ---- one pod, all nodes ----
    def score_pod(self, pod, outputs=True, out=None):
        """qs_score_pod: {"best"} and, with outputs, the per-node "feasible" / "scores" / "total"
        arrays (fresh copies, or the caller's reusable buffers from score_buffers() passed as
        `out`, filled in place).  outputs=False asks the library for the best node only."""
        p = np.array([pod], POD_DTYPE) if isinstance(pod, np.void) else pods_to_struct(pod)[:1]
        best = ctypes.c_int32(-2)
        if not outputs:
            self._chk(self.lib.qs_score_pod(self.ctx, _ptr(p), None, None, None, ctypes.byref(best)))
            return dict(best=best.value)
        if out is None:
            out = self.score_buffers()
        feas, score, total = out["feasible"], out["scores"], out["total"]
        if len(total) != self.n or score.shape != (self.n, 4) or feas.dtype != np.bool_:
            raise ValueError("score_pod: out buffers do not match the node table (use score_buffers())")
        self._chk(self.lib.qs_score_pod(self.ctx, _ptr(p), _ptr(feas), _ptr(score), _ptr(total),
                                        ctypes.byref(best)))
        return dict(feasible=feas, scores=score, total=total, best=best.value)

    def score_pod_packed(self, pod):
        """qs_score_pod_packed: (best, packed) with packed a copy of the n per-node words (0xFFFFFFFF
        = infeasible, else the four plugin scores as bytes, LeastAllocated in the low byte)."""
        p = np.array([pod], POD_DTYPE) if isinstance(pod, np.void) else pods_to_struct(pod)[:1]
        best = ctypes.c_int32(-2)
        ptr = ctypes.POINTER(ctypes.c_uint32)()
        self._chk(self.lib.qs_score_pod_packed(self.ctx, _ptr(p), ctypes.byref(ptr), ctypes.byref(best)))
        packed = np.ctypeslib.as_array(ptr, shape=(self.n,)).copy() if self.n and ptr else np.zeros(0, np.uint32)
        return best.value, packed

    def score_buffers(self):
        """Output arrays for score_pod(..., out=...) sized to the current table (feasible is a bool
        array the library fills with 0 / 1 bytes)."""
        return dict(feasible=np.zeros(self.n, np.bool_), scores=np.zeros((self.n, 4), np.int32),
                    total=np.zeros(self.n, np.int32))

    # ---- exact stream ----
    def schedule(self, pods, with_stats=False, mode="exact"):
        arr = pods_to_struct(pods)
        placement = np.empty(len(arr), np.int32)
        stats = QsStats()
        self._chk(self.lib.qs_schedule_stream(self.ctx, _ptr(arr), len(arr), MODES[mode],
                                              _ptr(placement), ctypes.byref(stats)))
        return (placement, stats.as_dict()) if with_stats else placement

    def prepare(self, pods):
        arr = pods_to_struct(pods)
        h = ctypes.c_void_p()
        self._chk(self.lib.qs_stream_prepare(self.ctx, _ptr(arr), len(arr), ctypes.byref(h)))
        return Stream(self, h, len(arr))


class Stream:
    """A prepared pod stream (device-resident pod records): run() is the timed device path."""

    def __init__(self, sched: Scheduler, handle, p):
        self.s, self.h, self.p = sched, handle, p
        self.stats = None

    def run(self, mode="exact"):
        """qs_stream_run: mode "exact" (spec S7/S8) or "batched" (spec S11)."""
        st = QsStats()
        self.s._chk(self.s.lib.qs_stream_run(self.s.ctx, self.h, MODES[mode], ctypes.byref(st)))
        self.stats = st.as_dict()
        return self.stats

    def results(self):
        placement = np.empty(self.p, np.int32)
        keys = np.empty(self.p, np.uint64)
        self.s._chk(self.s.lib.qs_stream_results(self.s.ctx, self.h, _ptr(placement), _ptr(keys)))
        return placement, keys

    def stamps(self):
        out = np.empty(self.p, np.uint64)
        self.s._chk(self.s.lib.qs_stream_stamps(self.s.ctx, self.h, _ptr(out)))
        return out

    def fit_errors(self, pods=None, by_taint=False):
        """qs_stream_fit_errors: per requested pod (arrival indices; default: every unschedulable
        pod) the count of nodes per FitError reason column (FIT_REASONS), against the table at that
        pod's turn.  Returns (indices, counts[m, 7]); with by_taint (qs_stream_fit_taints) also
        taint_counts[m, 64], the untolerated-taint column split by the node's first untolerated taint
        bit (upstream names that taint in the reason string)."""
        if pods is None:
            pl, _ = self.results()
            pods = np.nonzero(pl < 0)[0]
        idx = np.ascontiguousarray(pods, dtype=np.uint32)
        counts = np.zeros((len(idx), len(FIT_REASONS)), np.uint32)
        if not by_taint:
            self.s._chk(self.s.lib.qs_stream_fit_errors(self.s.ctx, self.h, _ptr(idx), len(idx), _ptr(counts)))
            return idx, counts
        tcounts = np.zeros((len(idx), 64), np.uint32)
        self.s._chk(self.s.lib.qs_stream_fit_taints(self.s.ctx, self.h, _ptr(idx), len(idx), _ptr(counts),
                                                     _ptr(tcounts)))
        return idx, counts, tcounts

    def free(self):
        if self.h:
            self.s._chk(self.s.lib.qs_stream_free(self.s.ctx, self.h))
            self.h = None


def dist_unique_id() -> bytes:
    """128-byte RCCL unique id (qs_dist_unique_id) for qs_open_shard; create on rank 0 only."""
    lib = load()
    buf = (ctypes.c_uint8 * 128)()
    st = lib.qs_dist_unique_id(buf)
    if st != QS_OK:
        raise QschedError(st, "qs_dist_unique_id failed")
    return bytes(buf)


def synth_generate(config: int, n: int, p: int, seed=None):
    """spec/synth.md cluster (host C++ generator in libqsched).  Returns (nodes dict, pods array)."""
    lib = load()
    nodes = empty_nodes(n)
    s, _ = _soa(nodes, lib_out=True)
    pods = np.zeros(p, POD_DTYPE)
    seed = 0x5EED0000 + config if seed is None else seed
    st = lib.qs_synth_generate(config, seed, n, p, ctypes.byref(s), _ptr(pods))
    if st != QS_OK:
        raise QschedError(st, "qs_synth_generate failed")
    return nodes, pods


def _containers(containers):
    arr = (QsContainer * max(1, len(containers)))()
    for i, c in enumerate(containers):
        for k, v in c.items():
            if k == "req_ext":
                for e, x in enumerate(v):
                    arr[i].req_ext[e] = int(x)
            elif k == "kind":
                arr[i].kind = {"regular": 0, "init": 1, "sidecar": 2}.get(v, v)
            elif k in ("req_cpu", "req_mem", "lim_cpu", "lim_mem"):
                setattr(arr[i], k, int(v))
                setattr(arr[i], "has_" + k, 1)
    return arr


def fit_error_message(counts, n_nodes, ext_names=("ext0", "ext1"), taint_counts=None, taint_names=None):
    """UP framework/types.go#FitError.Error() from one pod's reason counts: "0/N nodes are available:
    <count> <reason>, ..." with the "count reason" strings sorted as Go's sort.Strings does.

    Upstream's TaintToleration reason names the node's first untolerated taint ("node(s) had
    untolerated taint {key: value}", taint_toleration.go#Filter), so each distinct taint is its own
    reason.  Pass taint_counts (this pod's row of ``fit_errors(by_taint=True)``) and taint_names
    (interned bit -> "key: value", e.g. from qsched.workload's taint dictionary) to get that text;
    without them the untolerated-taint nodes are one reason and a bit without a name renders as
    "taint-<bit>"."""
    names = [r.format(ext0=ext_names[0], ext1=ext_names[1], taint="{taint}") for r in FIT_REASONS]
    parts = []
    for k, c in enumerate(counts):
        if not c:
            continue
        if k == QS_FIT_TAINT and taint_counts is not None:
            tc = np.asarray(taint_counts)
            assert int(tc.sum()) == int(c), "taint_counts must split this pod's untolerated-taint count"
            for b in np.nonzero(tc)[0]:
                nm = (taint_names or {}).get(int(b), f"taint-{int(b)}")
                parts.append(f"{int(tc[b])} " + names[k].replace("{taint}", nm))
        elif k == QS_FIT_TAINT:
            parts.append(f"{int(c)} node(s) had untolerated taint")
        else:
            parts.append(f"{int(c)} {names[k]}")
    parts.sort()
    msg = f"0/{n_nodes} nodes are available:"
    return msg + (f" {', '.join(parts)}." if parts else "")


def pod_from_containers(containers, overhead=None):
    """spec S2/S3 for a pod spec given as a list of container dicts (missing keys = missing)."""
    lib = load()
    arr = _containers(containers)
    out = np.zeros(1, POD_DTYPE)
    ov = None if overhead is None else (ctypes.c_int64 * 2)(*overhead)
    st = lib.qs_pod_from_containers(arr, len(containers), ov, _ptr(out))
    if st != QS_OK:
        raise QschedError(st, "qs_pod_from_containers failed")
    return out[0]


def compute_qos(containers) -> int:
    lib = load()
    return int(lib.qs_compute_qos(_containers(containers), len(containers)))
