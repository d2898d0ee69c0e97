"""Loader for libruserf_amd.so (the HIP/CDNA4 engine behind include/ruserf_amd.h).

There is deliberately no CPU fallback: if the shared library is missing or
fails to load, every engine call raises.  Build it with
`python -c "import __graft_entry__ as g; g.build()"` or `make -C ruserf_amd/csrc`.
"""
import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RSF_LIB_PATH") or os.path.join(HERE, "libruserf_amd.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "ruserf_amd.h")

RSF_OK = 0
RSF_ERR_DIM_MISMATCH = 1
RSF_ERR_INVALID_COORD = 2
RSF_ERR_INVALID_RTT = 3
RSF_ERR_ARG = -1
RSF_ERR_HIP = -2
RSF_ERR_NOMEM = -3
RSF_ERR_OVERFLOW = -4


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"ruserf_amd error {code}: {msg}")
        self.code = code


class RsfVivaldiXbufs(C.Structure):
    _fields_ = [("req_send", C.c_void_p), ("req_recv", C.c_void_p), ("rep_send", C.c_void_p),
                ("rep_recv", C.c_void_p), ("req_bucket_bytes", C.c_uint64), ("rep_bucket_bytes", C.c_uint64)]


class RsfCoordOpts(C.Structure):
    _fields_ = [("dimensionality", C.c_uint32), ("adjustment_window_size", C.c_uint32),
                ("latency_filter_size", C.c_uint32), ("_reserved", C.c_uint32),
                ("vivaldi_error_max", C.c_double), ("vivaldi_ce", C.c_double),
                ("vivaldi_cc", C.c_double), ("height_min", C.c_double),
                ("gravity_rho", C.c_double)]


_lib = None

P8 = C.POINTER(C.c_uint8)
P16 = C.POINTER(C.c_uint16)
P32 = C.POINTER(C.c_uint32)
PI32 = C.POINTER(C.c_int32)
P64 = C.POINTER(C.c_uint64)
PD = C.POINTER(C.c_double)
VP = C.c_void_p


def declared_symbols():
    """Function names declared in include/ruserf_amd.h."""
    with open(HEADER) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rsf_[a-z0-9_]+)\s*\(", src)))


def _sig(L, name, res, args):
    fn = getattr(L, name)
    fn.restype = res
    fn.argtypes = args


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineError(RSF_ERR_ARG, f"{LIB_PATH} not built: run __graft_entry__.build()")
    # torch-ROCm ships its own libamdhip64 (same SONAME, loaded by a different
    # file name): if ours initialised HIP first, torch would load a second
    # runtime and see no device.  Loading torch first makes libruserf_amd bind
    # to the runtime already in the process.  (The C ABI itself needs no torch.)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    i = C.c_int
    _sig(L, "rsf_last_error", C.c_char_p, [])
    _sig(L, "rsf_version", C.c_char_p, [])
    _sig(L, "rsf_device_count", i, [])
    _sig(L, "rsf_coord_opts_default", None, [C.POINTER(RsfCoordOpts)])
    _sig(L, "rsf_coord_row_stride", C.c_uint32, [C.c_uint32])
    _sig(L, "rsf_vivaldi_create", i, [C.POINTER(VP), C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32,
                                      C.POINTER(RsfCoordOpts), C.c_uint64, i])
    _sig(L, "rsf_vivaldi_destroy", i, [VP])
    _sig(L, "rsf_vivaldi_set_stream", i, [VP, VP])
    _sig(L, "rsf_vivaldi_sync", i, [VP])
    _sig(L, "rsf_vivaldi_get_coordinates", i, [VP, C.c_uint64, C.c_uint64, PD])
    _sig(L, "rsf_vivaldi_set_coordinate", i, [VP, C.c_uint64, PD, C.c_uint32, C.c_double, C.c_double,
                                              C.c_double])
    _sig(L, "rsf_vivaldi_forget_node", i, [VP, C.c_uint64, C.c_uint32])
    _sig(L, "rsf_vivaldi_resets", i, [VP, P64])
    _sig(L, "rsf_vivaldi_update_batch", i, [VP, P32, P32, PD, P32, P64, C.c_uint64, C.c_uint32, PI32, PD])
    _sig(L, "rsf_vivaldi_estimate_rtt_batch", i, [VP, P32, P32, C.c_uint64, P64])
    _sig(L, "rsf_vivaldi_estimate_rtt_device", i, [VP, VP, VP, C.c_uint64, VP])
    _sig(L, "rsf_vivaldi_round", i, [VP, C.c_uint32])
    _sig(L, "rsf_vivaldi_gen_probes", i, [VP, C.c_uint32, VP, VP])
    _sig(L, "rsf_vivaldi_observe", i, [VP, C.c_uint32, VP, VP, VP, C.c_uint32])
    _sig(L, "rsf_vivaldi_observe_range", i, [VP, C.c_uint32, VP, VP, VP, C.c_uint32, C.c_uint64, C.c_uint64])
    _sig(L, "rsf_vivaldi_flip", i, [VP])
    _sig(L, "rsf_vivaldi_table", i, [VP, C.POINTER(VP), P64])
    _sig(L, "rsf_vivaldi_true_rtt_ns", i, [VP, C.c_uint32, C.c_uint32, P64])
    _sig(L, "rsf_vivaldi_probe", i, [VP, C.c_uint32, VP, VP, VP, VP])
    _sig(L, "rsf_vivaldi_probe_acks", i, [VP, VP, VP, VP, VP, C.c_uint64])
    _sig(L, "rsf_vivaldi_exchange_buffers", i, [VP, C.c_uint32, C.POINTER(RsfVivaldiXbufs)])
    _sig(L, "rsf_vivaldi_exchange_requests", i, [VP, C.c_uint32, VP])
    _sig(L, "rsf_vivaldi_exchange_requests_range", i, [VP, C.c_uint32, VP, C.c_uint64, C.c_uint64])
    _sig(L, "rsf_vivaldi_exchange_serve", i, [VP, C.c_uint32])
    _sig(L, "rsf_vivaldi_exchange_apply", i, [VP, C.c_uint32])
    _sig(L, "rsf_vivaldi_exchange_status", i, [VP, C.POINTER(C.c_int)])
    try:
        from . import _gossip_sigs
        _gossip_sigs.declare(L)
    except ImportError:
        pass
    _lib = L
    return L


def check(rc):
    if rc != RSF_OK:
        raise EngineError(rc, lib().rsf_last_error().decode())
    return rc


def ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))
