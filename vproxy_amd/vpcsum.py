"""ctypes binding of libvpcsum.so (C-ABI in include/vpcsum.h) plus the host-side helpers the
vswitch mirror and the tests use.

There is deliberately NO CPU fallback: if the HIP library cannot be loaded, every entry point
raises :class:`VpcsumUnavailable`.  Device memory and streams come from PyTorch (plumbing only);
``import torch`` happens before the library is loaded so that libvpcsum binds to the same HIP
runtime instance as torch (both carry SONAME libamdhip64.so.7).
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

from .build import LIB

F_IP, F_L4, F_RAW, F_L4P, F_PRE = 0x01, 0x02, 0x04, 0x08, 0x10
S_IP_OK, S_L4_OK, S_UDP_NOCSUM, S_DONE, S_BAD_DESC = 0x01, 0x02, 0x04, 0x40, 0x80
S_TTL_EXPIRED = 0x20
MODE_COMPUTE, MODE_VERIFY, MODE_WRITE = 0x00, 0x01, 0x10
NAT_SRC, NAT_DST, NAT_SPORT, NAT_DPORT, NAT_DEC_TTL, NAT_SET_TTL = 0x01, 0x02, 0x04, 0x08, 0x10, 0x20
NAT_RFC1624, NAT_STRICT_JAVA = 0x00, 0x01
PRE_FMT_PRE4, PRE_FMT_PRE = 0, 1   # pre-image entries: NAT4_DTYPE (16 B, IPv4) / NAT_DTYPE (48 B)
PRE_HSUM = 0x80   # pre-image entry mask: the entry's first 8 bytes hold an HSUM_DTYPE record
ABI_VERSION = 4   # include/vpcsum.h VPCSUM_ABI_VERSION: the library this binding was written against
SYNTH_C1, SYNTH_C2, SYNTH_C3, SYNTH_C4, SYNTH_FUZZ, SYNTH_C5 = 1, 2, 3, 4, 5, 6

DESC_DTYPE = np.dtype([("l3_off", "<u8"), ("l3_len", "<u2"), ("l4_off", "<u2"), ("l3_ver", "u1"),
                       ("l4_proto", "u1"), ("flags", "u1"), ("rsv", "u1")])
NAT4_DTYPE = np.dtype([("src", "u1", 4), ("dst", "u1", 4), ("sport", "u1", 2), ("dport", "u1", 2),
                       ("mask", "u1"), ("rsv", "u1", 3)])
NAT_DTYPE = np.dtype([("src", "u1", 16), ("dst", "u1", 16), ("sport", "u1", 2), ("dport", "u1", 2),
                      ("mask", "u1"), ("ttl", "u1"), ("rsv", "u1", 10)])
NAT4R_DTYPE = np.dtype([("desc", DESC_DTYPE), ("rw", NAT4_DTYPE)])   # vpcsum_nat4_rec_t, 32 B
# vpcsum_tuple_t: the flow tuple of a parsed frame (network-order addresses and ports)
TUPLE_DTYPE = np.dtype([("src", "u1", 16), ("dst", "u1", 16), ("sport", "u1", 2), ("dport", "u1", 2),
                        ("l3_ver", "u1"), ("l4_proto", "u1"), ("tcp_flags", "u1"), ("rsv", "u1")])
# vpcsum_hsum_t: a received TCP / UDP frame's ingress header sum (l2_len 0: no record)
HSUM_DTYPE = np.dtype([("sum", "<u2"), ("l4_len", "<u2"), ("hlen", "u1"), ("l4_proto", "u1"), ("l3_ver", "u1"),
                       ("l2_len", "u1")])

# Every symbol include/vpcsum.h declares (tests check the .so exports all of them).
EXPORTS = [
    "vpcsum_abi_version", "vpcsum_last_error", "vpcsum_device_count", "vpcsum_set_device",
    "vpcsum_compute_async", "vpcsum_nat4_async", "vpcsum_nat_async", "vpcsum_parse_ether_async",
    "vpcsum_parse_ether_tuples_async", "vpcsum_read_probe_async",
    "vpcsum_pattern_probe_async", "vpcsum_nat4_pattern_probe_async", "vpcsum_nat4r_async",
    "vpcsum_nat4r_pattern_probe_async",
    "vpcsum_synth_async", "vpcsum_event_create", "vpcsum_event_destroy", "vpcsum_event_record",
    "vpcsum_event_elapsed_ms", "vpcsum_stream_sync", "vpcsum_ctx_create", "vpcsum_ctx_destroy",
    "vpcsum_ctx_register_arena", "vpcsum_ctx_unregister_arena", "vpcsum_ctx_submit", "vpcsum_ctx_wait",
    "vpcsum_ctx_pipeline", "vpcsum_ctx_set_service", "vpcsum_ctx_stats", "vpcsum_ctx_verify_frames",
    "vpcsum_ctx_parse_frames", "vpcsum_ctx_egress_frames", "Java_io_vproxy_vpcsum_VPCsum_egressFrames",
    "vpcsum_ctx_nat_submit", "Java_io_vproxy_vpcsum_VPCsum_natSubmit",
    "vpcsum_group_create", "vpcsum_group_create_list", "vpcsum_group_destroy", "vpcsum_group_register_arena",
    "vpcsum_group_unregister_arena", "vpcsum_group_submit", "vpcsum_group_wait", "vpcsum_group_nat_submit",
    "vpcsum_init", "vpcsum_shutdown", "vpcsum_register_arena", "vpcsum_batch_submit", "vpcsum_nat_submit",
    "vpcsum_batch_wait", "vpcsum_pre_async", "vpcsum_ctx_submit_pre", "vpcsum_group_submit_pre",
    "vpcsum_batch_submit_pre", "Java_io_vproxy_vpcsum_VPCsum_submitPre",
    "Java_io_vproxy_vpcsum_VPCsum_create", "Java_io_vproxy_vpcsum_VPCsum_registerArena",
    "Java_io_vproxy_vpcsum_VPCsum_submit", "Java_io_vproxy_vpcsum_VPCsum_waitFor",
    "Java_io_vproxy_vpcsum_VPCsum_close", "Java_io_vproxy_vpcsum_VPCsum_setService",
    "Java_io_vproxy_vpcsum_VPCsum_verifyFrames", "Java_io_vproxy_vpcsum_VPCsum_parseFrames",
    "vpcsum_ctx_verify_frames_hsum", "vpcsum_parse_ether_hsum_async", "Java_io_vproxy_vpcsum_VPCsum_verifyFramesHsum",
    "vpcsum_spin_probe_async", "vpcsum_pipe_create", "vpcsum_pipe_begin", "vpcsum_pipe_compute_async",
    "vpcsum_pipe_join", "vpcsum_pipe_destroy",
]


class VpcsumUnavailable(RuntimeError):
    pass


class VpcsumError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()

# Host ranges this binding page-locked (ptr -> nbytes, counted per registration) and the ranges it
# released since the last `released_ranges(clear=True)`: the GPU tests' audit checks that HIP no
# longer holds a released range as registered (tests/conftest.py, tests/hiputil.py).
_live_regs: dict[int, list[int]] = {}
_released: list[tuple[int, int]] = []
_leaked: list[dict] = []   # arrays of a context / group whose destroy failed: kept alive


# VPCSUM_AUDIT_REGISTRATIONS=1 (the GPU tests set it): right after each release, while the array
# is still referenced, ask HIP whether it still holds the range as page-locked; any that it does is
# recorded in _stale (a registration outliving its release: a later pageable copy from memory
# allocated at those addresses would go through its dead mapping).
_AUDIT = os.environ.get("VPCSUM_AUDIT_REGISTRATIONS") == "1"
_stale: list[tuple[int, int]] = []
_hip = None


class _PtrAttr(ctypes.Structure):   # hipPointerAttribute_t (hip_runtime_api.h)
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def hip_holds_registered(ptr: int) -> bool:
    """Whether the HIP runtime (the libamdhip64 this process loaded) holds host address `ptr` as
    page-locked memory (hipPointerGetAttributes: hipMemoryTypeHost)."""
    global _hip
    if _hip is None:
        lib()
        path = None
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64.so" in line:
                    path = line.split()[-1]
                    break
        if path is None:
            raise VpcsumUnavailable("libamdhip64 is not loaded")
        h = ctypes.CDLL(path)
        h.hipPointerGetAttributes.argtypes = [ctypes.POINTER(_PtrAttr), ctypes.c_void_p]
        h.hipPointerGetAttributes.restype = ctypes.c_int
        h.hipGetLastError.restype = ctypes.c_int
        _hip = h
    a = _PtrAttr()
    rc = _hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(ptr))
    _hip.hipGetLastError()   # an unknown pointer leaves hipErrorInvalidValue behind
    return rc == 0 and a.type == 1


def _reg_add(ptr: int, nbytes: int):
    with _lock:
        _live_regs.setdefault(ptr, []).append(nbytes)


def _reg_drop(ptr: int):
    with _lock:
        lst = _live_regs.get(ptr)
        if not lst:
            return
        n = lst.pop()
        _released.append((ptr, n))
        if not lst:
            del _live_regs[ptr]
        covered = any(q <= ptr < q + max(m) for q, m in _live_regs.items())
    if _AUDIT and not covered and any(hip_holds_registered(q) for q in _audit_points(ptr, n)):
        _stale.append((ptr, n))


def _audit_points(ptr: int, n: int, cap: int = 256) -> list[int]:
    """Addresses of a released range HIP is asked about: both ends and one address in every page
    between them (at most `cap`, evenly spread over a larger range)."""
    first, last = ptr, ptr + n - 1
    pages = (last >> 12) - (ptr >> 12) + 1
    step = max(1, -(-pages // cap))
    pts = [first, last]
    pts += [((ptr >> 12) + k) << 12 for k in range(1, pages - 1, step)]
    return pts


def released_ranges(clear: bool = True) -> list[tuple[int, int]]:
    """Ranges released (unregistered, or their context / group destroyed) that no registration of
    this binding covers any more."""
    with _lock:
        out = [(p, n) for p, n in _released
               if not any(q <= p < q + max(m) for q, m in _live_regs.items())]
        if clear:
            _released.clear()
        return out


def _declare(L):
    P, I, U8, U32, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint64
    sig = {
        "vpcsum_abi_version": ([], I),
        "vpcsum_last_error": ([], ctypes.c_char_p),
        "vpcsum_device_count": ([P], I),
        "vpcsum_set_device": ([I], I),
        "vpcsum_compute_async": ([P, U64, P, U32, P, P, U32, P], I),
        "vpcsum_nat4_async": ([P, U64, P, P, U32, P, U32, P], I),
        "vpcsum_nat4r_async": ([P, U64, P, U32, P, U32, P], I),
        "vpcsum_nat4r_pattern_probe_async": ([P, U64, P, U32, P], I),
        "vpcsum_nat_async": ([P, U64, P, P, U32, P, U32, P], I),
        "vpcsum_ctx_nat_submit": ([P, P, U64, P, P, U32, P, U32, P], I),
        "vpcsum_pre_async": ([P, U64, P, P, U32, U32, P, P, U32, P], I),
        "vpcsum_ctx_submit_pre": ([P, P, U64, P, P, U32, U32, P, P, U32, P], I),
        "vpcsum_group_submit_pre": ([P, P, U64, P, P, U32, U32, P, P, U32, P], I),
        "vpcsum_batch_submit_pre": ([P, U64, P, P, U32, U32, P, P, U32, P], I),
        "vpcsum_group_create": ([U64, U64, U32, P], I),
        "vpcsum_group_create_list": ([P, I, U64, U32, P], I),
        "vpcsum_group_destroy": ([P], I),
        "vpcsum_group_register_arena": ([P, P, U64], I),
        "vpcsum_group_unregister_arena": ([P, P], I),
        "vpcsum_group_submit": ([P, P, U64, P, U32, P, P, U32, P], I),
        "vpcsum_group_wait": ([P, U64], I),
        "vpcsum_group_nat_submit": ([P, P, U64, P, P, U32, P, U32, P], I),
        "vpcsum_init": ([U64, U64, U32], I),
        "vpcsum_shutdown": ([], I),
        "vpcsum_register_arena": ([P, U64], I),
        "vpcsum_batch_submit": ([P, U64, P, U32, P, P, U32, P], I),
        "vpcsum_nat_submit": ([P, U64, P, P, U32, P, U32, P], I),
        "vpcsum_batch_wait": ([U64], I),
        "vpcsum_parse_ether_async": ([P, U64, P, P, U32, U8, P, P, P], I),
        "vpcsum_parse_ether_tuples_async": ([P, U64, P, P, U32, U8, P, P, P, P], I),
        "vpcsum_parse_ether_hsum_async": ([P, U64, P, P, U32, U8, P, P, P, P], I),
        "vpcsum_read_probe_async": ([P, U64, P, U32, P], I),
        "vpcsum_pattern_probe_async": ([P, U64, P, U32, P, U32, P], I),
        "vpcsum_nat4_pattern_probe_async": ([P, U64, P, P, U32, P], I),
        "vpcsum_synth_async": ([P, U64, U32, U32, U32, U32, U64, U64, P, P], I),
        "vpcsum_event_create": ([P], I),
        "vpcsum_event_destroy": ([P], I),
        "vpcsum_event_record": ([P, P], I),
        "vpcsum_event_elapsed_ms": ([P, P, P], I),
        "vpcsum_stream_sync": ([P], I),
        "vpcsum_ctx_create": ([I, U64, U32, P], I),
        "vpcsum_ctx_destroy": ([P], I),
        "vpcsum_ctx_register_arena": ([P, P, U64], I),
        "vpcsum_ctx_unregister_arena": ([P, P], I),
        "vpcsum_ctx_set_service": ([P, U32], I),
        "vpcsum_ctx_stats": ([P, P, P], I),
        "vpcsum_ctx_verify_frames": ([P, P, U64, P, P, U32, P, P, P], I),
        "vpcsum_ctx_verify_frames_hsum": ([P, P, U64, P, P, U32, P, P, P, P], I),
        "vpcsum_pipe_create": ([P, P], I),
        "vpcsum_pipe_begin": ([P], I),
        "vpcsum_pipe_compute_async": ([P, P, U64, P, U32, P, P, U32], I),
        "vpcsum_pipe_join": ([P], I),
        "vpcsum_pipe_destroy": ([P], I),
        "vpcsum_spin_probe_async": ([U32, U32, U32, P], I),
        "vpcsum_ctx_parse_frames": ([P, P, U64, P, P, U32, P, P, P, P], I),
        "vpcsum_ctx_egress_frames": ([P, P, U64, P, P, P, U32, P, P, P], I),
        "vpcsum_ctx_submit": ([P, P, U64, P, U32, P, P, U32, P], I),
        "vpcsum_ctx_wait": ([P, U64], I),
        "vpcsum_ctx_pipeline": ([P, P, U32, U32, P, U32, P, U32, U32], I),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res


def lib():
    """Load libvpcsum.so (after torch, so both share one HIP runtime)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB):
                raise VpcsumUnavailable(f"{LIB} is missing: run `python -m vproxy_amd.build` "
                                        "(there is no CPU fallback)")
            try:
                import torch  # noqa: F401  -- bind torch's libamdhip64 first
            except ImportError:
                pass
            try:
                L = ctypes.CDLL(LIB)
            except OSError as e:
                raise VpcsumUnavailable(f"cannot load {LIB}: {e}") from e
            _declare(L)
            if L.vpcsum_abi_version() != ABI_VERSION:
                raise VpcsumUnavailable("ABI version mismatch")
            _lib = L
        return _lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = lib().vpcsum_last_error()
        raise VpcsumError(f"{what}: {msg.decode() if msg else rc}")


def _ptr(t) -> int | None:
    if t is None:
        return None
    if isinstance(t, np.ndarray):
        return t.ctypes.data
    return t.data_ptr()


def _stream(stream) -> int | None:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


# ------------------------------------------------------------------------------------------
# Device-resident API (torch CUDA tensors)
# ------------------------------------------------------------------------------------------
def compute(arena, desc, n: int | None = None, out=None, status=None, mode: int = MODE_COMPUTE,
            team_log2: int = 0, stream=None, plain_loads: bool = False, blocks_per_cu: int = 0,
            full_grid: bool = False):
    """Checksum a device-resident batch.  `arena` uint8 tensor, `desc` tensor holding n
    16-byte vpcsum_desc_t, `out` int32/uint32 tensor (n), `status` uint8 tensor (n)."""
    if n is None:
        n = desc.numel() * desc.element_size() // 16
    m = mode | ((team_log2 & 0x1F) << 8) | (((team_log2 >> 5) & 0x7) << 24) | (0x2000 if plain_loads else 0) | (0x4000 if full_grid else 0) | ((blocks_per_cu & 0xFF) << 16)
    _check(lib().vpcsum_compute_async(_ptr(arena), arena.numel(), _ptr(desc), n, _ptr(out), _ptr(status), m,
                                      _stream(stream)), "vpcsum_compute_async")


def nat4(arena, desc, rw, n: int, status=None, nat_mode: int = NAT_RFC1624, stream=None):
    _check(lib().vpcsum_nat4_async(_ptr(arena), arena.numel(), _ptr(desc), _ptr(rw), n, _ptr(status), nat_mode,
                                   _stream(stream)), "vpcsum_nat4_async")


def nat(arena, desc, rw, n: int, status=None, nat_mode: int = NAT_RFC1624, stream=None):
    """NAT / TTL rewrite with 48-B vpcsum_nat_t entries (IPv4 and IPv6): `rw` a uint8 tensor of n x 48."""
    _check(lib().vpcsum_nat_async(_ptr(arena), arena.numel(), _ptr(desc), _ptr(rw), n, _ptr(status), nat_mode,
                                  _stream(stream)), "vpcsum_nat_async")


def pre(arena, desc, pre_img, n: int, out=None, status=None, mode: int = MODE_WRITE, pre_fmt: int = PRE_FMT_PRE4,
        stream=None):
    """vpcsum_pre_async: the sums of the F_PRE descriptors from their pre-images (`pre_img`: n
    entries, NAT4_DTYPE bytes for PRE_FMT_PRE4 or NAT_DTYPE for PRE_FMT_PRE, holding the OLD
    addresses / ports); descriptors without F_PRE are left alone (run `compute` for them first)."""
    _check(lib().vpcsum_pre_async(_ptr(arena), arena.numel(), _ptr(desc), _ptr(pre_img), pre_fmt, n, _ptr(out),
                                  _ptr(status), mode, _stream(stream)), "vpcsum_pre_async")


def parse_ether(arena, frame_off, frame_len, n: int, desc, status=None, flags: int = F_IP | F_L4, stream=None,
                tuples=None, hsum=None):
    """Descriptors from raw frames on the GPU; with `tuples` (n x 40 bytes, TUPLE_DTYPE) also each
    frame's flow tuple (vpcsum_parse_ether_tuples_async); with `hsum` (n x 8 bytes, HSUM_DTYPE) each
    frame's ingress header sum instead (vpcsum_parse_ether_hsum_async)."""
    if hsum is not None:
        assert tuples is None and hsum.numel() * hsum.element_size() >= n * HSUM_DTYPE.itemsize
        _check(lib().vpcsum_parse_ether_hsum_async(_ptr(arena), arena.numel(), _ptr(frame_off), _ptr(frame_len), n,
                                                   flags, _ptr(desc), _ptr(status), _ptr(hsum), _stream(stream)),
               "vpcsum_parse_ether_hsum_async")
        return
    if tuples is None:
        _check(lib().vpcsum_parse_ether_async(_ptr(arena), arena.numel(), _ptr(frame_off), _ptr(frame_len), n, flags,
                                              _ptr(desc), _ptr(status), _stream(stream)), "vpcsum_parse_ether_async")
        return
    assert tuples.numel() * tuples.element_size() >= n * TUPLE_DTYPE.itemsize
    _check(lib().vpcsum_parse_ether_tuples_async(_ptr(arena), arena.numel(), _ptr(frame_off), _ptr(frame_len), n,
                                                 flags, _ptr(desc), _ptr(status), _ptr(tuples), _stream(stream)),
           "vpcsum_parse_ether_tuples_async")


def pattern_probe(arena, desc, n: int, sink, grid: int = 0, stream=None):
    """Read exactly the chunks the checksum kernel reads for `desc`, no checksum work (tooling)."""
    assert sink.numel() * sink.element_size() >= 4096, "sink needs 1024 words"
    _check(lib().vpcsum_pattern_probe_async(_ptr(arena), arena.numel(), _ptr(desc), n, _ptr(sink), grid,
                                            _stream(stream)), "vpcsum_pattern_probe_async")


def nat4r(arena, rec, n: int, status=None, nat_mode: int = NAT_RFC1624, stream=None):
    """vpcsum_nat4r_async: `rec` holds n NAT4R_DTYPE records (descriptor + IPv4 entry)."""
    _check(lib().vpcsum_nat4r_async(_ptr(arena), arena.numel(), _ptr(rec), n, _ptr(status), nat_mode, _stream(stream)),
           "vpcsum_nat4r_async")


def nat4r_pattern_probe(arena, rec, n: int, stream=None):
    _check(lib().vpcsum_nat4r_pattern_probe_async(_ptr(arena), arena.numel(), _ptr(rec), n, _stream(stream)),
           "vpcsum_nat4r_pattern_probe_async")


def nat4_pattern_probe(arena, desc, rw, n: int, stream=None):
    """NAT's memory operations for `desc` / `rw` (16-B entries) with no rewrite (tooling)."""
    _check(lib().vpcsum_nat4_pattern_probe_async(_ptr(arena), arena.numel(), _ptr(desc), _ptr(rw), n,
                                                 _stream(stream)), "vpcsum_nat4_pattern_probe_async")


def read_probe(buf, nbytes: int, sink, grid: int = 0, stream=None):
    _check(lib().vpcsum_read_probe_async(_ptr(buf), nbytes, _ptr(sink), grid, _stream(stream)),
           "vpcsum_read_probe_async")


def synth(arena, n: int, stride: int, l3_pad: int, workload: int, seed: int, first_index: int = 0,
          desc=None, stream=None):
    """arena None: the descriptors alone (desc required)."""
    _check(lib().vpcsum_synth_async(_ptr(arena) if arena is not None else None, arena.numel() if arena is not None else 0,
                                    n, stride, l3_pad, workload, seed, first_index, _ptr(desc), _stream(stream)),
           "vpcsum_synth_async")


class Pipe:
    """Two batches in flight on the device API (vpcsum_pipe_*): `begin()` forks the pipe's two
    streams from `stream`, `compute()` launches alternate between them (consecutive batches may run
    concurrently: their outputs must not overlap), `join()` makes `stream` wait for all of them."""

    def __init__(self, stream=None):
        h = ctypes.c_void_p()
        _check(lib().vpcsum_pipe_create(_stream(stream), ctypes.byref(h)), "vpcsum_pipe_create")
        self.h = h.value

    def begin(self):
        _check(lib().vpcsum_pipe_begin(self.h), "vpcsum_pipe_begin")

    def compute(self, arena, desc, n: int | None = None, out=None, status=None, mode: int = MODE_COMPUTE,
                team_log2: int = 0):
        if n is None:
            n = desc.numel() * desc.element_size() // 16
        m = mode | ((team_log2 & 0x1F) << 8) | (((team_log2 >> 5) & 0x7) << 24)
        _check(lib().vpcsum_pipe_compute_async(self.h, _ptr(arena), arena.numel(), _ptr(desc), n, _ptr(out),
                                               _ptr(status), m), "vpcsum_pipe_compute_async")

    def join(self):
        _check(lib().vpcsum_pipe_join(self.h), "vpcsum_pipe_join")

    def close(self):
        if self.h:
            lib().vpcsum_pipe_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Event:
    """HIP event recorded on an arbitrary (e.g. the kernel's) stream."""

    def __init__(self):
        h = ctypes.c_void_p()
        _check(lib().vpcsum_event_create(ctypes.byref(h)), "vpcsum_event_create")
        self.h = h.value

    def record(self, stream=None):
        _check(lib().vpcsum_event_record(self.h, _stream(stream)), "vpcsum_event_record")

    def elapsed_ms(self, end: "Event") -> float:
        ms = ctypes.c_float()
        _check(lib().vpcsum_event_elapsed_ms(self.h, end.h, ctypes.byref(ms)), "vpcsum_event_elapsed_ms")
        return ms.value

    def __del__(self):
        try:
            if _lib is not None and self.h:
                _lib.vpcsum_event_destroy(self.h)
        except Exception:
            pass


# ------------------------------------------------------------------------------------------
# Host-memory API (what the Java binding drives)
# ------------------------------------------------------------------------------------------
class Context:
    def __init__(self, device: int = 0, max_arena: int = 1 << 26, max_pkts: int = 1 << 16):
        h = ctypes.c_void_p()
        _check(lib().vpcsum_ctx_create(device, max_arena, max_pkts, ctypes.byref(h)), "vpcsum_ctx_create")
        self.h = h.value
        # numpy buffers the library holds raw pointers to: registered arrays (until unregister /
        # close) and the buffers of the batch in flight on each of the context's two slots
        self._pinned = {}
        self._inflight = {}

    def register(self, arr: np.ndarray):
        _check(lib().vpcsum_ctx_register_arena(self.h, arr.ctypes.data, arr.nbytes), "vpcsum_ctx_register_arena")
        self._pinned[arr.ctypes.data] = arr
        _reg_add(arr.ctypes.data, arr.nbytes)

    def unregister(self, arr: np.ndarray):
        _check(lib().vpcsum_ctx_unregister_arena(self.h, arr.ctypes.data), "vpcsum_ctx_unregister_arena")
        self._pinned.pop(arr.ctypes.data, None)
        _reg_drop(arr.ctypes.data)

    def submit(self, arena: np.ndarray, desc: np.ndarray, out: np.ndarray | None, status: np.ndarray | None = None,
               mode: int = MODE_COMPUTE) -> int:
        """out None: no out words (a verify whose result is the status bytes)."""
        t = ctypes.c_uint64()
        _check(lib().vpcsum_ctx_submit(self.h, arena.ctypes.data, arena.nbytes, desc.ctypes.data, len(desc),
                                       None if out is None else out.ctypes.data,
                                       None if status is None else status.ctypes.data, mode,
                                       ctypes.byref(t)), "vpcsum_ctx_submit")
        self._inflight[t.value & 1] = (arena, desc, out, status)
        return t.value

    def wait(self, ticket: int):
        _check(lib().vpcsum_ctx_wait(self.h, ticket), "vpcsum_ctx_wait")

    def submit_pre(self, arena: np.ndarray, desc: np.ndarray, pre_img: np.ndarray, out: np.ndarray,
                   status: np.ndarray | None = None, mode: int = MODE_COMPUTE) -> int:
        """vpcsum_ctx_submit_pre: F_PRE descriptors take their L4 sum from pre_img[i] (NAT_DTYPE or
        NAT4_DTYPE entries, old values), the others are summed in full; one submission."""
        fmt = PRE_FMT_PRE if pre_img.dtype == NAT_DTYPE else PRE_FMT_PRE4
        assert pre_img.dtype in (NAT_DTYPE, NAT4_DTYPE) and len(pre_img) >= len(desc)
        t = ctypes.c_uint64()
        _check(lib().vpcsum_ctx_submit_pre(self.h, arena.ctypes.data, arena.nbytes, desc.ctypes.data,
                                           pre_img.ctypes.data, fmt, len(desc), out.ctypes.data,
                                           None if status is None else status.ctypes.data, mode, ctypes.byref(t)),
               "vpcsum_ctx_submit_pre")
        self._inflight[t.value & 1] = (arena, desc, pre_img, out, status)
        return t.value

    def run_pre(self, arena, desc, pre_img, mode: int = MODE_COMPUTE):
        out = np.zeros(len(desc), np.uint32)
        status = np.zeros(len(desc), np.uint8)
        self.wait(self.submit_pre(arena, desc, pre_img, out, status, mode))
        return out, status

    def verify_frames(self, arena: np.ndarray, frame_off: np.ndarray, frame_len: np.ndarray, sums: bool = True):
        """Ingress verify of received Ethernet frames in a registered arena: parsed and verified
        on the GPU in one submission.  Returns (out, status) per frame; sums=False: (None, status),
        the kernel writes no out words (GpuCsumBatch.verifyFrames' form)."""
        n = len(frame_off)
        fo = np.ascontiguousarray(frame_off, dtype=np.uint64)
        fl = np.ascontiguousarray(frame_len, dtype=np.uint32)
        out = np.zeros(n, np.uint32) if sums else None
        status = np.zeros(n, np.uint8)
        t = ctypes.c_uint64()
        _check(lib().vpcsum_ctx_verify_frames(self.h, arena.ctypes.data, arena.nbytes, fo.ctypes.data, fl.ctypes.data,
                                              n, None if out is None else out.ctypes.data, status.ctypes.data,
                                              ctypes.byref(t)),
               "vpcsum_ctx_verify_frames")
        self.wait(t.value)
        return out, status

    def verify_frames_hsum(self, arena: np.ndarray, frame_off: np.ndarray, frame_len: np.ndarray):
        """verify_frames(sums=False) that also records each frame's ingress header sum
        (vpcsum_ctx_verify_frames_hsum, GpuCsumBatch.verifyFrames' form since ABI 4).  Returns
        (status, hsum): S_* bytes and HSUM_DTYPE records per frame."""
        n = len(frame_off)
        fo = np.ascontiguousarray(frame_off, dtype=np.uint64)
        fl = np.ascontiguousarray(frame_len, dtype=np.uint32)
        status = np.zeros(n, np.uint8)
        hsum = np.zeros(n, HSUM_DTYPE)
        t = ctypes.c_uint64()
        _check(lib().vpcsum_ctx_verify_frames_hsum(self.h, arena.ctypes.data, arena.nbytes, fo.ctypes.data,
                                                   fl.ctypes.data, n, None, status.ctypes.data, hsum.ctypes.data,
                                                   ctypes.byref(t)), "vpcsum_ctx_verify_frames_hsum")
        self.wait(t.value)
        return status, hsum

    def parse_frames(self, arena: np.ndarray, frame_off: np.ndarray, frame_len: np.ndarray):
        """Batched parse of received Ethernet frames in a registered arena, with flow tuples
        (vpcsum_ctx_parse_frames).  Returns (descriptors, status, tuples) per frame."""
        n = len(frame_off)
        fo = np.ascontiguousarray(frame_off, dtype=np.uint64)
        fl = np.ascontiguousarray(frame_len, dtype=np.uint32)
        desc = np.zeros(n, DESC_DTYPE)
        status = np.zeros(n, np.uint8)
        tuples = np.zeros(n, TUPLE_DTYPE)
        t = ctypes.c_uint64()
        _check(lib().vpcsum_ctx_parse_frames(self.h, arena.ctypes.data, arena.nbytes, fo.ctypes.data, fl.ctypes.data,
                                             n, desc.ctypes.data, status.ctypes.data, tuples.ctypes.data,
                                             ctypes.byref(t)), "vpcsum_ctx_parse_frames")
        self.wait(t.value)
        return desc, status, tuples

    def egress_frames(self, arena: np.ndarray, frame_off: np.ndarray, frame_len: np.ndarray,
                      frame_flags: np.ndarray):
        """Egress flush of frames in a registered arena, each with its own F_* flags: parsed on
        the GPU and written in place in one submission (vpcsum_ctx_egress_frames).  Returns
        (out, status) per frame; S_BAD_DESC = refused, nothing written."""
        n = len(frame_off)
        fo = np.ascontiguousarray(frame_off, dtype=np.uint64)
        fl = np.ascontiguousarray(frame_len, dtype=np.uint32)
        ff = np.ascontiguousarray(frame_flags, dtype=np.uint8)
        out = np.zeros(n, np.uint32)
        status = np.zeros(n, np.uint8)
        t = ctypes.c_uint64()
        _check(lib().vpcsum_ctx_egress_frames(self.h, arena.ctypes.data, arena.nbytes, fo.ctypes.data, fl.ctypes.data,
                                              ff.ctypes.data, n, out.ctypes.data, status.ctypes.data,
                                              ctypes.byref(t)), "vpcsum_ctx_egress_frames")
        self.wait(t.value)
        return out, status

    def nat_submit(self, arena: np.ndarray, desc: np.ndarray, rw: np.ndarray, status: np.ndarray | None = None,
                   nat_mode: int = NAT_RFC1624) -> int:
        """NAT / TTL rewrites of host frames (vpcsum_ctx_nat_submit); rw: NAT_DTYPE entries."""
        assert rw.dtype == NAT_DTYPE and len(rw) >= len(desc)
        t = ctypes.c_uint64()
        _check(lib().vpcsum_ctx_nat_submit(self.h, arena.ctypes.data, arena.nbytes, desc.ctypes.data,
                                           rw.ctypes.data, len(desc), None if status is None else status.ctypes.data,
                                           nat_mode, ctypes.byref(t)), "vpcsum_ctx_nat_submit")
        self._inflight[t.value & 1] = (arena, desc, rw, status)
        return t.value

    def nat(self, arena: np.ndarray, desc: np.ndarray, rw: np.ndarray, nat_mode: int = NAT_RFC1624) -> np.ndarray:
        status = np.zeros(len(desc), np.uint8)
        self.wait(self.nat_submit(arena, desc, rw, status, nat_mode))
        return status

    def set_service(self, idle_us: int):
        """Low-latency flushes from registered arenas (persistent service grid); 0 = off."""
        _check(lib().vpcsum_ctx_set_service(self.h, idle_us), "vpcsum_ctx_set_service")

    def stats(self) -> dict:
        b, n = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().vpcsum_ctx_stats(self.h, ctypes.byref(b), ctypes.byref(n)), "vpcsum_ctx_stats")
        return {"service_batches": b.value, "service_launches": n.value}

    def run(self, arena, desc, mode: int = MODE_COMPUTE):
        out = np.zeros(len(desc), np.uint32)
        status = np.zeros(len(desc), np.uint8)
        self.wait(self.submit(arena, desc, out, status, mode))
        return out, status

    def pipeline(self, arena: np.ndarray, stride: int, copy_bytes: int, desc: np.ndarray, out: np.ndarray,
                 mode: int = MODE_COMPUTE, chunks: int = 8):
        _check(lib().vpcsum_ctx_pipeline(self.h, arena.ctypes.data, stride, copy_bytes, desc.ctypes.data, len(desc),
                                         out.ctypes.data, mode, chunks), "vpcsum_ctx_pipeline")

    def close(self):
        """Destroy the context (its batches finish, its page-locks go).  If an unregister failed,
        the arrays it held stay referenced (never freed while HIP may still map them) and the error
        is raised."""
        if self.h:
            rc = lib().vpcsum_ctx_destroy(self.h)
            self.h = None
            if rc != 0:
                _leaked.append(self._pinned.copy())
                _check(rc, "vpcsum_ctx_destroy")
            for p in self._pinned:
                _reg_drop(p)
            self._pinned.clear()
            self._inflight.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Group:
    """Several GPUs behind one host batch (vpcsum_group_*): the batch is cut by bytes into one
    contiguous range per device.  `devices` may repeat a device (several contexts on one GPU)."""

    def __init__(self, devices=(0,), max_arena: int = 1 << 26, max_pkts: int = 1 << 16):
        h = ctypes.c_void_p()
        arr = (ctypes.c_int * len(devices))(*devices)
        _check(lib().vpcsum_group_create_list(arr, len(devices), max_arena, max_pkts, ctypes.byref(h)),
               "vpcsum_group_create_list")
        self.h = h.value
        self._pinned = {}
        self._inflight = {}

    def register(self, arr: np.ndarray):
        _check(lib().vpcsum_group_register_arena(self.h, arr.ctypes.data, arr.nbytes), "vpcsum_group_register_arena")
        self._pinned[arr.ctypes.data] = arr
        _reg_add(arr.ctypes.data, arr.nbytes)

    def unregister(self, arr: np.ndarray):
        _check(lib().vpcsum_group_unregister_arena(self.h, arr.ctypes.data), "vpcsum_group_unregister_arena")
        self._pinned.pop(arr.ctypes.data, None)
        _reg_drop(arr.ctypes.data)

    def submit(self, arena: np.ndarray, desc: np.ndarray, out: np.ndarray, status: np.ndarray | None = None,
               mode: int = MODE_COMPUTE) -> int:
        t = ctypes.c_uint64()
        _check(lib().vpcsum_group_submit(self.h, arena.ctypes.data, arena.nbytes, desc.ctypes.data, len(desc),
                                         out.ctypes.data, None if status is None else status.ctypes.data, mode,
                                         ctypes.byref(t)), "vpcsum_group_submit")
        self._inflight[t.value & 1] = (arena, desc, out, status)
        return t.value

    def submit_pre(self, arena: np.ndarray, desc: np.ndarray, pre_img: np.ndarray, out: np.ndarray,
                   status: np.ndarray | None = None, mode: int = MODE_COMPUTE) -> int:
        """vpcsum_group_submit_pre: Context.submit_pre cut over the group's devices."""
        fmt = PRE_FMT_PRE if pre_img.dtype == NAT_DTYPE else PRE_FMT_PRE4
        assert pre_img.dtype in (NAT_DTYPE, NAT4_DTYPE) and len(pre_img) >= len(desc)
        t = ctypes.c_uint64()
        _check(lib().vpcsum_group_submit_pre(self.h, arena.ctypes.data, arena.nbytes, desc.ctypes.data,
                                             pre_img.ctypes.data, fmt, len(desc), out.ctypes.data,
                                             None if status is None else status.ctypes.data, mode, ctypes.byref(t)),
               "vpcsum_group_submit_pre")
        self._inflight[t.value & 1] = (arena, desc, pre_img, out, status)
        return t.value

    def nat_submit(self, arena: np.ndarray, desc: np.ndarray, rw: np.ndarray, status: np.ndarray | None = None,
                   nat_mode: int = NAT_RFC1624) -> int:
        """NAT / TTL rewrites of host frames cut over the group's devices (vpcsum_group_nat_submit)."""
        assert rw.dtype == NAT_DTYPE and len(rw) >= len(desc)
        t = ctypes.c_uint64()
        _check(lib().vpcsum_group_nat_submit(self.h, arena.ctypes.data, arena.nbytes, desc.ctypes.data,
                                             rw.ctypes.data, len(desc), None if status is None else status.ctypes.data,
                                             nat_mode, ctypes.byref(t)), "vpcsum_group_nat_submit")
        self._inflight[t.value & 1] = (arena, desc, rw, status)
        return t.value

    def wait(self, ticket: int):
        _check(lib().vpcsum_group_wait(self.h, ticket), "vpcsum_group_wait")

    def run(self, arena, desc, mode: int = MODE_COMPUTE):
        out = np.zeros(len(desc), np.uint32)
        status = np.zeros(len(desc), np.uint8)
        self.wait(self.submit(arena, desc, out, status, mode))
        return out, status

    def close(self):
        if self.h:
            rc = lib().vpcsum_group_destroy(self.h)
            self.h = None
            if rc != 0:
                _leaked.append(self._pinned.copy())
                _check(rc, "vpcsum_group_destroy")
            for p in self._pinned:
                _reg_drop(p)
            self._pinned.clear()
            self._inflight.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def desc_to_tensor(desc: np.ndarray, device="cuda"):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(desc).view(np.uint8).copy())
    # through page-locked memory: no pageable host-to-device copy of an array whose addresses a
    # context may have registered and unregistered before (DESIGN_HISTORY.md "Round 5: experiments")
    return (t.pin_memory() if str(device).startswith("cuda") else t).to(device)


def tensor_to_desc(t) -> np.ndarray:
    return t.cpu().numpy().view(DESC_DTYPE).copy()
