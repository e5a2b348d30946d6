"""ctypes binding of libdraid_ec.so (the C ABI in include/draid_ec.h).

Plumbing for tests and bench.py: it passes raw device pointers (from torch
tensors or draid_ec_device_alloc) straight to the C ABI -- no torch types cross
the boundary.  There is no fallback: if the shared library is missing or the GPU
is unusable every call raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
# DRAID_EC_LIB selects another build of the same ABI (tools: the lab build with
# kernel variants, `make -C draid-spdk_amd lab`).
LIB_PATH = os.environ.get("DRAID_EC_LIB") or os.path.join(HERE, "libdraid_ec.so")
LAB_LIB_PATH = os.path.join(HERE, "liblab", "libdraid_ec.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "draid_ec.h")

FAIL_NONE = 0xFF
PQ_CHECK_STATIC_MAX_VECTS = 257  # DRAID_PQ_CHECK_STATIC_MAX_VECTS

# Every symbol include/draid_ec.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "draid_xor_gen", "draid_pq_gen", "draid_xor_check", "draid_pq_check",
    "draid_gf_mul", "draid_gf_inv", "draid_gf_vect_mul_init", "draid_gf_vect_mul",
    "draid_recover", "draid_ec_encode", "draid_ec_reconstruct",
    "draid_ec_abi_version", "draid_ec_last_error", "draid_ec_set_device",
    "draid_ec_device_count", "draid_ec_stream_create", "draid_ec_stream_destroy",
    "draid_ec_stream_query", "draid_ec_stream_synchronize", "draid_ec_device_alloc",
    "draid_ec_device_free", "draid_ec_host_register", "draid_ec_host_unregister",
    "draid_ec_memcpy_async", "draid_ec_ctx_create", "draid_ec_ctx_destroy",
    "draid_ec_ctx_stream", "draid_ec_ctx_encode_sg", "draid_ec_ctx_reconstruct_sg",
    "draid_ec_ctx_flush", "draid_ec_ctx_query", "draid_ec_ctx_synchronize",
    "draid_ec_ctx_queued", "draid_ec_host_encode", "draid_ec_host_reconstruct",
    "draid_ec_encode_strided", "draid_ec_reconstruct_strided",
    "draid_ec_ctx_update_sg", "draid_ec_host_device_pointer", "draid_ec_ctx_set_autoflush",
    "draid_pq_check_static", "draid_ec_reconstruct_status",
    "draid_ec_reconstruct_strided_status", "draid_ec_device_pointer",
    "draid_ec_pointer_cache_flush", "draid_ec_ctx_flush_ticket", "draid_ec_ctx_ticket_query",
    "draid_ec_ctx_set_host_pointers", "draid_ec_host_alloc", "draid_ec_host_free",
    "draid_ec_ctx_discard_queued", "draid_ec_device_current",
    "draid_ec_ctx_mark", "draid_ec_ctx_rollback", "draid_ec_ctx_fence",
    "draid_ec_shard_of", "draid_ec_shard_range", "draid_ec_shard_count",
    "draid_ec_mgpu_create", "draid_ec_mgpu_destroy", "draid_ec_mgpu_devices",
    "draid_ec_mgpu_device", "draid_ec_mgpu_stream", "draid_ec_mgpu_encode",
    "draid_ec_mgpu_reconstruct", "draid_ec_mgpu_encode_strided",
    "draid_ec_mgpu_reconstruct_strided", "draid_ec_mgpu_query", "draid_ec_mgpu_synchronize",
)

SHARD_RANGE, SHARD_MOD = 0, 1


class HostStripes(C.Structure):
    _fields_ = [("k", C.c_uint32), ("m", C.c_uint32), ("strip_len", C.c_uint64),
                ("nstripes", C.c_uint32), ("flags", C.c_uint32), ("base", C.c_void_p),
                ("strip_stride", C.c_uint64), ("stripe_stride", C.c_uint64)]


class IoVec(C.Structure):
    _fields_ = [("iov_base", C.c_void_p), ("iov_len", C.c_size_t)]


class StripeBatch(C.Structure):
    _fields_ = [
        ("k", C.c_uint32),
        ("m", C.c_uint32),
        ("strip_len", C.c_uint64),
        ("nstripes", C.c_uint32),
        ("flags", C.c_uint32),
        ("strips", C.c_void_p),
    ]


class DraidError(RuntimeError):
    pass


def build(force: bool = False) -> str:
    """Compile libdraid_ec.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    if force or not os.path.exists(LIB_PATH):
        target = "lab" if os.path.abspath(LIB_PATH) == LAB_LIB_PATH else "libdraid_ec.so"
        subprocess.check_call(["make", "-s", "-C", HERE, target])
    return LIB_PATH


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DraidError(f"{LIB_PATH} is missing: run `make -C {HERE}` (no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        i32, vp, u8 = C.c_int, C.c_void_p, C.c_ubyte
        for f in ("draid_xor_gen", "draid_pq_gen", "draid_xor_check", "draid_pq_check"):
            getattr(L, f).argtypes = [i32, i32, C.POINTER(vp)]
            getattr(L, f).restype = i32
        L.draid_pq_check_static.argtypes = [i32, i32, C.POINTER(vp), vp, vp]
        L.draid_pq_check_static.restype = i32
        L.draid_gf_mul.argtypes = [u8, u8]
        L.draid_gf_mul.restype = u8
        L.draid_gf_inv.argtypes = [u8]
        L.draid_gf_inv.restype = u8
        L.draid_gf_vect_mul_init.argtypes = [u8, vp]
        L.draid_gf_vect_mul.argtypes = [i32, vp, vp, vp]
        L.draid_recover.argtypes = [i32, i32, i32, C.POINTER(vp), i32, C.POINTER(i32)]
        L.draid_ec_encode.argtypes = [C.POINTER(StripeBatch), vp]
        L.draid_ec_reconstruct.argtypes = [C.POINTER(StripeBatch), vp, vp]
        L.draid_ec_reconstruct_status.argtypes = [C.POINTER(StripeBatch), vp, vp, vp]
        L.draid_ec_reconstruct_strided_status.argtypes = [C.POINTER(HostStripes), vp, vp, vp]
        L.draid_ec_device_pointer.argtypes = [vp, C.c_size_t, C.POINTER(vp)]
        L.draid_ec_pointer_cache_flush.restype = None
        L.draid_ec_last_error.restype = C.c_char_p
        L.draid_ec_set_device.argtypes = [i32]
        L.draid_ec_device_count.argtypes = [C.POINTER(i32)]
        L.draid_ec_device_current.argtypes = [C.POINTER(i32)]
        L.draid_ec_stream_create.argtypes = [C.POINTER(vp)]
        for f in ("draid_ec_stream_destroy", "draid_ec_stream_query",
                  "draid_ec_stream_synchronize", "draid_ec_device_free",
                  "draid_ec_host_unregister"):
            getattr(L, f).argtypes = [vp]
        L.draid_ec_device_alloc.argtypes = [C.POINTER(vp), C.c_size_t]
        L.draid_ec_host_register.argtypes = [vp, C.c_size_t]
        L.draid_ec_host_alloc.argtypes = [C.POINTER(vp), C.c_size_t]
        L.draid_ec_host_free.argtypes = [vp]
        L.draid_ec_ctx_discard_queued.argtypes = [vp]
        u64 = C.c_uint64
        L.draid_ec_shard_of.argtypes = [u64, u64, i32, i32]
        L.draid_ec_shard_range.argtypes = [u64, i32, i32, C.POINTER(u64), C.POINTER(u64)]
        L.draid_ec_shard_count.argtypes = [u64, i32, i32, i32]
        L.draid_ec_shard_count.restype = u64
        L.draid_ec_mgpu_create.argtypes = [C.POINTER(vp), i32, C.POINTER(i32)]
        for f in ("draid_ec_mgpu_destroy", "draid_ec_mgpu_devices", "draid_ec_mgpu_query",
                  "draid_ec_mgpu_synchronize"):
            getattr(L, f).argtypes = [vp]
        L.draid_ec_mgpu_device.argtypes = [vp, i32]
        L.draid_ec_mgpu_stream.argtypes = [vp, i32]
        L.draid_ec_mgpu_stream.restype = vp
        L.draid_ec_mgpu_encode.argtypes = [vp, C.POINTER(StripeBatch)]
        L.draid_ec_mgpu_reconstruct.argtypes = [vp, C.POINTER(StripeBatch), C.POINTER(vp),
                                                C.POINTER(vp)]
        L.draid_ec_mgpu_encode_strided.argtypes = [vp, C.POINTER(HostStripes)]
        L.draid_ec_mgpu_reconstruct_strided.argtypes = [vp, C.POINTER(HostStripes), C.POINTER(vp),
                                                        C.POINTER(vp)]
        L.draid_ec_host_device_pointer.argtypes = [vp, C.POINTER(vp)]
        L.draid_ec_memcpy_async.argtypes = [vp, vp, C.c_size_t, i32, vp]
        L.draid_ec_set_variant.argtypes = [i32]
        L.draid_ec_ctx_create.argtypes = [C.POINTER(vp)]
        for f in ("draid_ec_ctx_destroy", "draid_ec_ctx_flush", "draid_ec_ctx_query",
                  "draid_ec_ctx_synchronize", "draid_ec_ctx_mark", "draid_ec_ctx_rollback",
                  "draid_ec_ctx_fence"):
            getattr(L, f).argtypes = [vp]
        L.draid_ec_ctx_stream.argtypes = [vp]
        L.draid_ec_ctx_stream.restype = vp
        L.draid_ec_ctx_queued.argtypes = [vp]
        L.draid_ec_ctx_queued.restype = C.c_uint64
        L.draid_ec_ctx_set_autoflush.argtypes = [vp, C.c_uint64]
        L.draid_ec_ctx_flush_ticket.argtypes = [vp, C.POINTER(C.c_uint64)]
        L.draid_ec_ctx_ticket_query.argtypes = [vp, C.c_uint64]
        L.draid_ec_ctx_set_host_pointers.argtypes = [vp, i32]
        L.draid_ec_ctx_test_fail_after.argtypes = [vp, i32]
        L.draid_ec_ctx_test_fail_after.restype = None
        L.draid_ec_ctx_test_staged.argtypes = [vp]
        L.draid_ec_ctx_test_staged.restype = i32
        L.draid_ec_test_launch_events.argtypes = [vp, vp]
        L.draid_ec_test_launch_events.restype = None
        L.draid_ec_test_event_create.argtypes = [C.POINTER(vp)]
        L.draid_ec_test_event_destroy.argtypes = [vp]
        L.draid_ec_test_event_elapsed_ms.argtypes = [vp, vp, C.POINTER(C.c_float)]
        L.draid_ec_ctx_encode_sg.argtypes = [vp, C.c_uint32, C.c_uint32, vp, vp, vp, C.c_size_t]
        L.draid_ec_ctx_reconstruct_sg.argtypes = [vp, C.c_uint32, C.c_uint32, vp, vp, vp,
                                                  C.c_size_t, i32, vp]
        L.draid_ec_ctx_update_sg.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp,
                                             vp, vp, vp, vp, C.c_size_t]
        L.draid_ec_encode_strided.argtypes = [C.POINTER(HostStripes), vp]
        L.draid_ec_reconstruct_strided.argtypes = [C.POINTER(HostStripes), vp, vp]
        L.draid_ec_host_encode.argtypes = [C.POINTER(HostStripes), C.c_uint32]
        L.draid_ec_host_reconstruct.argtypes = [C.POINTER(HostStripes), vp, C.c_uint32]
        _lib = L
    return _lib


# ---- measurement hooks (not part of the C ABI of the header) ----

def event_create() -> int:
    ev = C.c_void_p()
    _check(lib().draid_ec_test_event_create(C.byref(ev)), "event_create")
    return ev.value


def event_destroy(ev: int) -> None:
    lib().draid_ec_test_event_destroy(ev)


def event_elapsed_ms(start: int, stop: int) -> float:
    ms = C.c_float()
    _check(lib().draid_ec_test_event_elapsed_ms(start, stop, C.byref(ms)), "event_elapsed_ms")
    return float(ms.value)


def launch_events(start: int, stop: int) -> None:
    """The next batched launch of this thread stamps `start` and `stop` from its own dispatch
    (no event packets around it)."""
    lib().draid_ec_test_launch_events(start, stop)


def last_error() -> str:
    return lib().draid_ec_last_error().decode()


def _check(rc: int, what: str) -> int:
    if rc < 0:
        raise DraidError(f"{what} failed ({rc}): {last_error()}")
    return rc


def _ptr(x) -> int:
    return x if isinstance(x, int) else x.data_ptr()


def _array(ptrs) -> C.Array:
    return (C.c_void_p * len(ptrs))(*[_ptr(p) for p in ptrs])


# ---- isa-l-shaped synchronous calls (device pointers) ----

def xor_gen(ptrs, length: int) -> int:
    return _check(lib().draid_xor_gen(len(ptrs), length, _array(ptrs)), "xor_gen")


def pq_gen(ptrs, length: int) -> int:
    return _check(lib().draid_pq_gen(len(ptrs), length, _array(ptrs)), "pq_gen")


def xor_check(ptrs, length: int) -> int:
    return _check(lib().draid_xor_check(len(ptrs), length, _array(ptrs)), "xor_check")


def pq_check(ptrs, length: int) -> int:
    return _check(lib().draid_pq_check(len(ptrs), length, _array(ptrs)), "pq_check")


def pq_check_static(ptrs, length: int, result_ptr, stream: int) -> int:
    """Allocation-free draid_pq_check: enqueues on `stream`, verdict to *result_ptr."""
    return _check(lib().draid_pq_check_static(len(ptrs), length, _array(ptrs), _ptr(result_ptr),
                                              stream), "pq_check_static")


def gf_mul(a: int, b: int) -> int:
    return lib().draid_gf_mul(a, b)


def gf_inv(a: int) -> int:
    return lib().draid_gf_inv(a)


def gf_vect_mul_init(c: int) -> bytes:
    buf = (C.c_ubyte * 32)()
    lib().draid_gf_vect_mul_init(c, buf)
    return bytes(buf)


def gf_vect_mul(length: int, tbl: bytes, src, dst) -> int:
    t = (C.c_ubyte * 32)(*tbl)
    return _check(lib().draid_gf_vect_mul(length, t, _ptr(src), _ptr(dst)), "gf_vect_mul")


def recover(k: int, m: int, length: int, ptrs, fail) -> int:
    f = (C.c_int * max(1, len(fail)))(*fail)
    return _check(lib().draid_recover(k, m, length, _array(ptrs), len(fail), f), "recover")


# ---- batched asynchronous API ----

def make_batch(k: int, m: int, strip_len: int, nstripes: int, table_ptr) -> StripeBatch:
    return StripeBatch(k, m, strip_len, nstripes, 0, _ptr(table_ptr))


def encode(batch: StripeBatch, stream: int) -> int:
    return _check(lib().draid_ec_encode(C.byref(batch), stream), "ec_encode")


def reconstruct(batch: StripeBatch, fail_ptr, stream: int) -> int:
    return _check(lib().draid_ec_reconstruct(C.byref(batch), _ptr(fail_ptr), stream),
                  "ec_reconstruct")


def reconstruct_status(batch: StripeBatch, fail_ptr, counter_ptr, stream: int) -> int:
    return _check(lib().draid_ec_reconstruct_status(C.byref(batch), _ptr(fail_ptr),
                                                    _ptr(counter_ptr), stream),
                  "ec_reconstruct_status")


def device_pointer(ptr: int, nbytes: int):
    """Address a kernel may use for [ptr, ptr + nbytes), or None (pageable host memory)."""
    d = C.c_void_p()
    rc = _check(lib().draid_ec_device_pointer(ptr, nbytes, C.byref(d)), "device_pointer")
    return None if rc else d.value


def stream_create() -> int:
    s = C.c_void_p()
    _check(lib().draid_ec_stream_create(C.byref(s)), "stream_create")
    return s.value


def stream_destroy(stream: int) -> None:
    _check(lib().draid_ec_stream_destroy(stream), "stream_destroy")


def stream_query(stream: int) -> int:
    return _check(lib().draid_ec_stream_query(stream), "stream_query")


def stream_synchronize(stream: int) -> None:
    _check(lib().draid_ec_stream_synchronize(stream), "stream_synchronize")


# ---- host memory ----

def host_register(ptr: int, nbytes: int) -> None:
    _check(lib().draid_ec_host_register(ptr, nbytes), "host_register")


def host_unregister(ptr: int) -> None:
    _check(lib().draid_ec_host_unregister(ptr), "host_unregister")


def host_device_pointer(ptr: int):
    """Device address of a registered / pinned host byte, or None."""
    d = C.c_void_p()
    rc = _check(lib().draid_ec_host_device_pointer(ptr, C.byref(d)), "host_device_pointer")
    return None if rc else d.value


# ---- host-resident stripes ----

def encode_strided(base, k, m, strip_len, nstripes, strip_stride, stripe_stride,
                   stream: int) -> int:
    d = HostStripes(k, m, strip_len, nstripes, 0, _ptr(base), strip_stride, stripe_stride)
    return _check(lib().draid_ec_encode_strided(C.byref(d), stream), "encode_strided")


def reconstruct_strided(base, k, m, strip_len, nstripes, strip_stride, stripe_stride, fail,
                        stream: int, counter=None) -> int:
    d = HostStripes(k, m, strip_len, nstripes, 0, _ptr(base), strip_stride, stripe_stride)
    if counter is not None:
        return _check(lib().draid_ec_reconstruct_strided_status(C.byref(d), _ptr(fail),
                                                                _ptr(counter), stream),
                      "reconstruct_strided_status")
    return _check(lib().draid_ec_reconstruct_strided(C.byref(d), _ptr(fail), stream),
                  "reconstruct_strided")


HOST_STAGED = 1


def host_encode(base, k, m, strip_len, nstripes, strip_stride, stripe_stride, chunk=0,
                flags=0) -> int:
    h = HostStripes(k, m, strip_len, nstripes, flags, _ptr(base), strip_stride, stripe_stride)
    return _check(lib().draid_ec_host_encode(C.byref(h), chunk), "host_encode")


def host_reconstruct(base, k, m, strip_len, nstripes, strip_stride, stripe_stride, fail,
                     chunk=0, flags=0) -> int:
    h = HostStripes(k, m, strip_len, nstripes, flags, _ptr(base), strip_stride, stripe_stride)
    return _check(lib().draid_ec_host_reconstruct(C.byref(h), _ptr(fail), chunk),
                  "host_reconstruct")


# ---- scatter-gather context ----

class Ctx:
    """Owns a draid_ec_ctx (one stream + descriptor ring); single-threaded."""

    def __init__(self):
        h = C.c_void_p()
        _check(lib().draid_ec_ctx_create(C.byref(h)), "ctx_create")
        self.h = h.value

    def close(self):
        if self.h:
            lib().draid_ec_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _lists(strips):
        """strips: list (k+m) of lists of (ptr, len) runs."""
        arrs = [(IoVec * max(1, len(s)))(*[IoVec(_ptr(p), n) for p, n in s]) for s in strips]
        heads = (C.c_void_p * len(strips))(*[C.addressof(a) for a in arrs])
        cnts = (C.c_int * len(strips))(*[len(s) for s in strips])
        return arrs, heads, cnts

    def encode_sg(self, k, m, strips, length, offsets=None):
        arrs, heads, cnts = self._lists(strips)
        off = (C.c_size_t * len(strips))(*offsets) if offsets else None
        return _check(lib().draid_ec_ctx_encode_sg(self.h, k, m, heads, cnts, off, length),
                      "ctx_encode_sg")

    def reconstruct_sg(self, k, m, strips, length, fail, offsets=None):
        arrs, heads, cnts = self._lists(strips)
        off = (C.c_size_t * len(strips))(*offsets) if offsets else None
        f = (C.c_int * max(1, len(fail)))(*fail)
        return _check(lib().draid_ec_ctx_reconstruct_sg(self.h, k, m, heads, cnts, off, length,
                                                        len(fail), f), "ctx_reconstruct_sg")

    def update_sg(self, k, m, data_idx, old, new, parity, length):
        """old/new: per touched chunk lists of (ptr, len) runs; parity: [P runs, (Q runs)]."""
        oa, oh, oc = self._lists(old)
        na, nh, nc = self._lists(new)
        pa, ph, pc = self._lists(parity)
        idx = (C.c_int * len(data_idx))(*data_idx)
        return _check(lib().draid_ec_ctx_update_sg(self.h, k, m, len(data_idx), idx, oh, oc, nh,
                                                   nc, ph, pc, length), "ctx_update_sg")

    def flush(self):
        return _check(lib().draid_ec_ctx_flush(self.h), "ctx_flush")

    def query(self):
        return _check(lib().draid_ec_ctx_query(self.h), "ctx_query")

    def synchronize(self):
        return _check(lib().draid_ec_ctx_synchronize(self.h), "ctx_synchronize")

    def queued(self):
        return lib().draid_ec_ctx_queued(self.h)

    def mark(self) -> int:
        return _check(lib().draid_ec_ctx_mark(self.h), "ctx_mark")

    def rollback(self) -> int:
        return _check(lib().draid_ec_ctx_rollback(self.h), "ctx_rollback")

    def fence(self) -> int:
        return _check(lib().draid_ec_ctx_fence(self.h), "ctx_fence")

    def flush_ticket(self) -> int:
        t = C.c_uint64()
        _check(lib().draid_ec_ctx_flush_ticket(self.h, C.byref(t)), "ctx_flush_ticket")
        return t.value

    def ticket_query(self, ticket: int) -> int:
        return _check(lib().draid_ec_ctx_ticket_query(self.h, ticket), "ctx_ticket_query")

    def set_host_pointers(self, on: bool):
        return _check(lib().draid_ec_ctx_set_host_pointers(self.h, int(on)), "ctx_set_host_pointers")

    def test_fail_after(self, n: int):
        """Test hook: the n-th descriptor piece launched from now on fails."""
        lib().draid_ec_ctx_test_fail_after(self.h, n)

    def test_staged(self) -> int:
        """Test hook: descriptor pieces uploaded ahead of the flush, not yet launched."""
        return lib().draid_ec_ctx_test_staged(self.h)

    def set_autoflush(self, segments: int):
        return _check(lib().draid_ec_ctx_set_autoflush(self.h, segments), "ctx_set_autoflush")


# ---- several GPUs from one process ----

def shard_of(stripe: int, nstripes: int, ndevices: int, policy: int = SHARD_RANGE) -> int:
    return lib().draid_ec_shard_of(stripe, nstripes, ndevices, policy)


def shard_range(nstripes: int, ndevices: int, device: int):
    lo, hi = C.c_uint64(), C.c_uint64()
    rc = lib().draid_ec_shard_range(nstripes, ndevices, device, C.byref(lo), C.byref(hi))
    if rc:
        raise DraidError(last_error())
    return lo.value, hi.value


def shard_count(nstripes: int, ndevices: int, device: int, policy: int = SHARD_RANGE) -> int:
    return lib().draid_ec_shard_count(nstripes, ndevices, device, policy)


class MultiGpu:
    """draid_ec_mgpu: a stream per device slot, every call fans out over the slots."""

    def __init__(self, devices=None):
        h = C.c_void_p()
        n = len(devices) if devices is not None else 0
        arr = (C.c_int * n)(*devices) if devices is not None else None
        _check(lib().draid_ec_mgpu_create(C.byref(h), n, arr), "mgpu_create")
        self.h = h.value
        self.n = lib().draid_ec_mgpu_devices(self.h)

    def close(self):
        if self.h:
            lib().draid_ec_mgpu_destroy(self.h)
            self.h = None

    def device(self, slot):
        return lib().draid_ec_mgpu_device(self.h, slot)

    def stream(self, slot):
        return lib().draid_ec_mgpu_stream(self.h, slot)

    def encode(self, batches):
        arr = (StripeBatch * self.n)(*batches)
        return _check(lib().draid_ec_mgpu_encode(self.h, arr), "mgpu_encode")

    def reconstruct(self, batches, fails, counters=None):
        arr = (StripeBatch * self.n)(*batches)
        f = (C.c_void_p * self.n)(*[_ptr(x) if x is not None else None for x in fails])
        c = (C.c_void_p * self.n)(*[_ptr(x) for x in counters]) if counters else None
        return _check(lib().draid_ec_mgpu_reconstruct(self.h, arr, f, c), "mgpu_reconstruct")

    def query(self):
        return _check(lib().draid_ec_mgpu_query(self.h), "mgpu_query")

    def synchronize(self):
        return _check(lib().draid_ec_mgpu_synchronize(self.h), "mgpu_synchronize")


def set_variant(v: int) -> None:
    lib().draid_ec_set_variant(v)
