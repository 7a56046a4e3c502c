"""ctypes mirror of include/qsched.h (the C ABI of libqsched.so).

The struct layouts below are checked against the library at load time (``qs_struct_size``); a
mismatch raises instead of silently corrupting memory.  The library is loaded from the package
directory (built in-tree by ``make -C custom-k8s-scheduler_amd``); there is no fallback path — a
missing library raises ``QschedLibraryMissing``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# QSCHED_LIB (diagnostic builds, e.g. tools/diag_build.sh) overrides the in-tree library
LIB_PATH = os.environ.get("QSCHED_LIB") or os.path.join(PKG_ROOT, "libqsched.so")

QS_ABI_VERSION = 3
QS_MAX_EXT = 2
QS_MAX_TERMS = 4
QS_MAX_APPS = 1024
QS_MAX_ZONES = 64
QS_AA_NONE, QS_AA_HOSTNAME, QS_AA_ZONE = 0, 1, 2
QS_MAX_SCORE_RES = 4
# qs_fit_reason: FitError reason columns of qs_stream_fit_errors, with upstream's reason strings
FIT_REASONS = ["Too many pods", "Insufficient cpu", "Insufficient memory", "Insufficient {ext0}",
               "Insufficient {ext1}", "node(s) had untolerated taint {{{taint}}}",
               "node(s) didn't match Pod's node affinity/selector"]
QS_FIT_TAINT = 5
# qs_resource: scoring-resource ids ("ext0" / "ext1" = the table's extended-resource columns)
RESOURCES = {"cpu": 1, "memory": 2, "ext0": 3, "ext1": 4}

QS_OK, QS_EINVAL, QS_EDEVICE, QS_ETIMEOUT, QS_ENOMEM, QS_ESTATE = range(6)
STATUS_NAMES = {0: "QS_OK", 1: "QS_EINVAL", 2: "QS_EDEVICE", 3: "QS_ETIMEOUT", 4: "QS_ENOMEM",
                5: "QS_ESTATE"}
QS_QOS_BESTEFFORT, QS_QOS_BURSTABLE, QS_QOS_GUARANTEED = 0, 1, 2
QS_MODE_EXACT, QS_MODE_BATCHED = 0, 1
ENGINES = {"auto": 0, "persistent": 1, "scan": 2, "lookahead": 3, "batched": 4, "allreduce": 5}
ENGINE_NAMES = {v: k for k, v in ENGINES.items()}
LAYOUT_NAMES = {0: "compact", 1: "wide"}


class QschedLibraryMissing(RuntimeError):
    pass


class QschedError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class QsConfig(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_uint32), ("engine", ctypes.c_int32),
                ("fit_weight_cpu", ctypes.c_int64), ("fit_weight_mem", ctypes.c_int64),
                ("w_fit", ctypes.c_int32 * 3), ("w_bal", ctypes.c_int32 * 3),
                ("w_taint", ctypes.c_int32), ("w_affinity", ctypes.c_int32),
                ("enable_taint", ctypes.c_int32), ("enable_affinity", ctypes.c_int32),
                ("balanced_skip_besteffort", ctypes.c_int32), ("qos_sort", ctypes.c_int32),
                ("lookahead", ctypes.c_int32), ("record_timestamps", ctypes.c_int32),
                ("profile_kernels", ctypes.c_int32), ("virtual_shards", ctypes.c_int32),
                ("lookahead_serial", ctypes.c_int32),
                ("scan_soa_min_nodes", ctypes.c_int32), ("batch_pods", ctypes.c_int32),
                ("n_fit_resources", ctypes.c_int32), ("fit_resources", (ctypes.c_int32 * 2) * QS_MAX_SCORE_RES),
                ("n_balanced_resources", ctypes.c_int32),
                ("balanced_resources", ctypes.c_int32 * QS_MAX_SCORE_RES),
                ("reserved", ctypes.c_int32 * 3)]


_NODE_COLS = ["alloc_cpu", "alloc_mem", "alloc_ext", "max_pods", "req_cpu", "req_mem", "req_ext",
              "nz_cpu", "nz_mem", "pods", "taint_hard", "taint_soft", "label_bits", "zone"]


class QsNodeSoa(ctypes.Structure):
    _fields_ = [(f, ctypes.c_void_p) for f in _NODE_COLS]


class QsNodeRow(ctypes.Structure):
    _fields_ = [("alloc_cpu", ctypes.c_int64), ("alloc_mem", ctypes.c_int64),
                ("alloc_ext", ctypes.c_int64 * QS_MAX_EXT), ("max_pods", ctypes.c_int64),
                ("req_cpu", ctypes.c_int64), ("req_mem", ctypes.c_int64),
                ("req_ext", ctypes.c_int64 * QS_MAX_EXT), ("nz_cpu", ctypes.c_int64),
                ("nz_mem", ctypes.c_int64), ("pods", ctypes.c_int64),
                ("taint_hard", ctypes.c_uint64), ("taint_soft", ctypes.c_uint64),
                ("label_bits", ctypes.c_uint64 * 2), ("zone", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class QsContainer(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("has_req_cpu", ctypes.c_int32),
                ("has_req_mem", ctypes.c_int32), ("has_lim_cpu", ctypes.c_int32),
                ("has_lim_mem", ctypes.c_int32), ("req_cpu", ctypes.c_int64),
                ("req_mem", ctypes.c_int64), ("lim_cpu", ctypes.c_int64),
                ("lim_mem", ctypes.c_int64), ("req_ext", ctypes.c_int64 * QS_MAX_EXT)]


class QsStats(ctypes.Structure):
    _fields_ = [("pods", ctypes.c_uint64), ("placed", ctypes.c_uint64),
                ("unschedulable", ctypes.c_uint64), ("evals", ctypes.c_uint64),
                ("batches", ctypes.c_uint64), ("truncations", ctypes.c_uint64),
                ("wall_s", ctypes.c_double), ("h2d_s", ctypes.c_double), ("d2h_s", ctypes.c_double),
                ("p50_cycle_us", ctypes.c_double), ("p99_cycle_us", ctypes.c_double),
                ("max_cycle_us", ctypes.c_double), ("engine_used", ctypes.c_int32),
                ("table_layout", ctypes.c_int32), ("resumed_windows", ctypes.c_uint64),
                ("device_faults", ctypes.c_uint64),
                ("resident", ctypes.c_int32), ("reserved", ctypes.c_int32), ("kernel_s", ctypes.c_double * 4),
                ("kernel_launches", ctypes.c_uint64 * 4)]

    KERNELS = ("persistent", "scan", "select", "resolve")

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_
             if f not in ("reserved", "kernel_s", "kernel_launches")}
        d["engine_used"] = ENGINE_NAMES.get(self.engine_used, self.engine_used)
        d["table_layout"] = LAYOUT_NAMES.get(self.table_layout, self.table_layout)
        d["kernels"] = {k: {"s": self.kernel_s[i], "launches": int(self.kernel_launches[i])}
                        for i, k in enumerate(self.KERNELS) if self.kernel_launches[i]}
        return d


# qs_pod as a numpy structured dtype (C layout, 248 bytes)
POD_DTYPE = np.dtype([
    ("req_cpu", "<i8"), ("req_mem", "<i8"), ("req_ext", "<i8", (QS_MAX_EXT,)),
    ("nz_cpu", "<i8"), ("nz_mem", "<i8"), ("qos", "<i4"), ("priority", "<i4"),
    ("tol_hard", "<u8"), ("tol_soft", "<u8"), ("sel", "<u8", (2,)),
    ("n_req_terms", "<i4"), ("n_pref_terms", "<i4"),
    ("req_terms", "<u8", (QS_MAX_TERMS, 2)), ("pref_terms", "<u8", (QS_MAX_TERMS, 2)),
    ("pref_weight", "<i4", (QS_MAX_TERMS,)), ("app", "<i4"), ("anti_affinity", "<i4"),
], align=True)

_P = ctypes.c_void_p
_SIGS = {
    "qs_config_default": (None, [_P]),
    "qs_open": (ctypes.c_int, [_P, ctypes.c_int, _P]),
    "qs_open_shard": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P]),
    "qs_dist_unique_id": (ctypes.c_int, [_P]),
    "qs_dist_mailbox_export": (ctypes.c_int, [_P, _P]),
    "qs_dist_mailbox_connect": (ctypes.c_int, [_P, _P]),
    "qs_close": (ctypes.c_int, [_P]),
    "qs_last_error": (ctypes.c_char_p, [_P]),
    "qs_version": (ctypes.c_char_p, []),
    "qs_nodes_load": (ctypes.c_int, [_P, _P, ctypes.c_uint32]),
    "qs_nodes_read": (ctypes.c_int, [_P, _P, ctypes.c_uint32]),
    "qs_node_upsert": (ctypes.c_int, [_P, ctypes.c_uint32, _P, ctypes.c_uint64]),
    "qs_table_save": (ctypes.c_int, [_P]),
    "qs_table_restore": (ctypes.c_int, [_P]),
    "qs_reserve": (ctypes.c_int, [_P, ctypes.c_uint32, _P]),
    "qs_unreserve": (ctypes.c_int, [_P, ctypes.c_uint32, _P]),
    "qs_score_pod": (ctypes.c_int, [_P, _P, _P, _P, _P, _P]),
    "qs_score_pod_packed": (ctypes.c_int, [_P, _P, _P, _P]),
    "qs_schedule_stream": (ctypes.c_int, [_P, _P, ctypes.c_uint32, ctypes.c_int, _P, _P]),
    "qs_stream_prepare": (ctypes.c_int, [_P, _P, ctypes.c_uint32, _P]),
    "qs_stream_run": (ctypes.c_int, [_P, _P, ctypes.c_int, _P]),
    "qs_stream_results": (ctypes.c_int, [_P, _P, _P, _P]),
    "qs_stream_stamps": (ctypes.c_int, [_P, _P, _P]),
    "qs_stream_fit_errors": (ctypes.c_int, [_P, _P, _P, ctypes.c_uint32, _P]),
    "qs_stream_fit_taints": (ctypes.c_int, [_P, _P, _P, ctypes.c_uint32, _P, _P]),
    "qs_stream_free": (ctypes.c_int, [_P, _P]),
    "qs_pod_from_containers": (ctypes.c_int, [_P, ctypes.c_uint32, _P, _P]),
    "qs_compute_qos": (ctypes.c_int32, [_P, ctypes.c_uint32]),
    "qs_synth_generate": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32,
                                         ctypes.c_uint32, _P, _P]),
    "qs_struct_size": (ctypes.c_size_t, [ctypes.c_int]),
}
EXPORTED = sorted(_SIGS)

_LIB = None


def load(path: str = LIB_PATH):
    """Load libqsched.so and bind every C-ABI symbol.  Raises if the library is missing."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise QschedLibraryMissing(
            f"{path} not found: build it with `make -C custom-k8s-scheduler_amd` (hipcc, gfx950)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    expect = {0: ctypes.sizeof(QsConfig), 1: ctypes.sizeof(QsNodeSoa), 2: ctypes.sizeof(QsNodeRow),
              3: POD_DTYPE.itemsize, 4: ctypes.sizeof(QsContainer), 5: ctypes.sizeof(QsStats)}
    for k, v in expect.items():
        got = lib.qs_struct_size(k)
        if got != v:
            raise RuntimeError(f"ABI struct {k} size mismatch: C {got} vs Python {v}")
    _LIB = lib
    return lib
