"""ctypes loader for the C oracle (``liboracle.so``) -- TEST INFRASTRUCTURE ONLY.

The oracle restates isa-l v2.30.0's xor_gen / pq_gen / gf_* semantics and the
reference's recovery formulas on the CPU (see ``isal_oracle.h`` for the
citations).  Only tests/, ``__graft_entry__.smoke()`` and bench.py's
``cpu_baseline`` leg may import this package; the product library under
``draid-spdk_amd/`` never touches it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


def build(force: bool = False) -> str:
    srcs = [os.path.join(HERE, f) for f in ("isal_oracle.c", "isal_simd.c", "bdevperf_raid5.c", "isal_oracle.h")]
    if force or not os.path.exists(LIB_PATH) or \
            os.path.getmtime(LIB_PATH) < max(os.path.getmtime(f) for f in srcs):
        subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    return LIB_PATH


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        u8, i32, sz, u32, vp = C.c_ubyte, C.c_int, C.c_size_t, C.c_uint32, C.c_void_p
        L.orc_gf_mul.restype = u8
        L.orc_gf_mul.argtypes = [u8, u8]
        L.orc_gf_inv.restype = u8
        L.orc_gf_inv.argtypes = [u8]
        L.orc_gf_pow2.restype = u8
        L.orc_gf_pow2.argtypes = [i32]
        L.orc_gf_tables.argtypes = [vp, vp]
        L.orc_gf_vect_mul_init.argtypes = [u8, vp]
        L.orc_gf_vect_mul.argtypes = [i32, vp, vp, vp]
        for f in ("orc_xor_gen", "orc_pq_gen", "orc_xor_check", "orc_pq_check"):
            getattr(L, f).argtypes = [i32, i32, C.POINTER(vp)]
            getattr(L, f).restype = i32
        L.orc_recover.argtypes = [i32, i32, i32, C.POINTER(vp), i32, C.POINTER(i32)]
        L.orc_encode_strided.argtypes = [i32, i32, sz, u32, vp, sz, sz]
        L.orc_recover_strided.argtypes = [i32, i32, sz, u32, vp, sz, sz, vp]
        L.orc_bench_encode_reconstruct.restype = C.c_double
        L.orc_bench_encode_reconstruct.argtypes = [i32, i32, sz, u32, vp, sz, sz, vp, i32, i32,
                                                   C.c_double, C.POINTER(C.c_uint64)]
        L.orc_bench_encode_reconstruct_impl.restype = C.c_double
        L.orc_bench_encode_reconstruct_impl.argtypes = [i32, i32, i32, sz, u32, vp, sz, sz, vp,
                                                        i32, i32, C.c_double,
                                                        C.POINTER(C.c_uint64)]
        L.orc_simd_xor_gen.argtypes = [i32, i32, C.POINTER(vp)]
        L.orc_simd_encode_strided.argtypes = [i32, i32, sz, u32, vp, sz, sz]
        L.orc_simd_recover_strided.argtypes = [i32, i32, sz, u32, vp, sz, sz, vp]
        L.orc_raid5_parity_chunk.argtypes = [i32, i32, C.c_uint64]
        L.orc_raid5_data_chunk_to_disk.argtypes = [i32, i32]
        P64 = C.POINTER(C.c_uint64)
        L.orc_raid5_start_geometry.argtypes = [i32, i32, C.c_uint64, u32, P64, P64, P64, P64]
        L.orc_srand.argtypes = [C.c_uint]
        L.orc_rand_buffer.argtypes = [vp, C.c_long]
        L.orc_glibc_srand.argtypes = [C.c_uint]
        L.orc_glibc_rand_buffer.argtypes = [vp, C.c_long]
        L.orc_fill_splitmix.argtypes = [vp, sz, C.c_uint64]
        L.orc_fill_ut_ref_pattern.argtypes = [vp, C.c_uint64, u32]
        L.orc_bdevperf_raid5_fsw.restype = C.c_double
        L.orc_bdevperf_raid5_fsw.argtypes = [i32, sz, sz, i32, C.c_double, C.POINTER(C.c_uint64),
                                             C.POINTER(C.c_ubyte)]
        _lib = L
    return _lib


def _ptrs(rows: list[np.ndarray]):
    arr = (C.c_void_p * len(rows))(*[r.ctypes.data for r in rows])
    return arr


def xor_gen(vects: list[np.ndarray], length: int) -> int:
    return lib().orc_xor_gen(len(vects), length, _ptrs(vects))


def pq_gen(vects: list[np.ndarray], length: int) -> int:
    return lib().orc_pq_gen(len(vects), length, _ptrs(vects))


def xor_check(vects: list[np.ndarray], length: int) -> int:
    return lib().orc_xor_check(len(vects), length, _ptrs(vects))


def pq_check(vects: list[np.ndarray], length: int) -> int:
    return lib().orc_pq_check(len(vects), length, _ptrs(vects))


def recover(vects: list[np.ndarray], k: int, m: int, length: int, fail: list[int]) -> int:
    f = (C.c_int * max(1, len(fail)))(*fail)
    return lib().orc_recover(k, m, length, _ptrs(vects), len(fail), f)


def gf_mul(a: int, b: int) -> int:
    return lib().orc_gf_mul(a, b)


def gf_inv(a: int) -> int:
    return lib().orc_gf_inv(a)


def gf_pow2(e: int) -> int:
    return lib().orc_gf_pow2(e)


def gf_tables() -> tuple[np.ndarray, np.ndarray]:
    e = np.zeros(256, np.uint8)
    g = np.zeros(256, np.uint8)
    lib().orc_gf_tables(e.ctypes.data, g.ctypes.data)
    return e, g


def gf_vect_mul_init(c: int) -> np.ndarray:
    t = np.zeros(32, np.uint8)
    lib().orc_gf_vect_mul_init(c, t.ctypes.data)
    return t


def gf_vect_mul(length: int, tbl: np.ndarray, src: np.ndarray, dst: np.ndarray) -> int:
    return lib().orc_gf_vect_mul(length, tbl.ctypes.data, src.ctypes.data, dst.ctypes.data)


def encode_strided(buf: np.ndarray, k: int, m: int, length: int, nstripes: int,
                   strip_stride: int, stripe_stride: int) -> int:
    return lib().orc_encode_strided(k, m, length, nstripes, buf.ctypes.data, strip_stride,
                                    stripe_stride)


def recover_strided(buf: np.ndarray, k: int, m: int, length: int, nstripes: int,
                    strip_stride: int, stripe_stride: int, fail: np.ndarray) -> int:
    fail = np.ascontiguousarray(fail, dtype=np.uint8)
    return lib().orc_recover_strided(k, m, length, nstripes, buf.ctypes.data, strip_stride,
                                     stripe_stride, fail.ctypes.data)


def raid5_parity_chunk(n: int, max_degraded: int, stripe_index: int) -> int:
    return lib().orc_raid5_parity_chunk(n, max_degraded, stripe_index)


def raid5_data_chunk_to_disk(parity_chunk: int, data_idx: int) -> int:
    return lib().orc_raid5_data_chunk_to_disk(parity_chunk, data_idx)


def raid5_start_geometry(n: int, max_degraded: int, min_blockcnt: int, strip_size: int):
    out = [C.c_uint64() for _ in range(4)]
    lib().orc_raid5_start_geometry(n, max_degraded, min_blockcnt, strip_size,
                                   *[C.byref(o) for o in out])
    return tuple(o.value for o in out)


def srand(seed: int) -> None:
    lib().orc_srand(seed)


def rand_buffer(n: int) -> np.ndarray:
    b = np.zeros(n, np.uint8)
    lib().orc_rand_buffer(b.ctypes.data, n)
    return b


def glibc_srand(seed: int) -> None:
    lib().orc_glibc_srand(seed)


def glibc_rand_buffer(n: int) -> np.ndarray:
    b = np.zeros(n, np.uint8)
    lib().orc_glibc_rand_buffer(b.ctypes.data, n)
    return b


def fill_splitmix(n: int, seed: int) -> np.ndarray:
    b = np.zeros(n, np.uint8)
    lib().orc_fill_splitmix(b.ctypes.data, n, seed)
    return b


def ut_ref_pattern(num_blocks: int, blocklen: int) -> np.ndarray:
    b = np.zeros(num_blocks * blocklen, np.uint8)
    lib().orc_fill_ut_ref_pattern(b.ctypes.data, num_blocks, blocklen)
    return b


def simd_available() -> bool:
    return bool(lib().orc_simd_available())


def simd_xor_gen(vects: list[np.ndarray], length: int) -> int:
    return lib().orc_simd_xor_gen(len(vects), length, _ptrs(vects))


def simd_encode_strided(buf: np.ndarray, k: int, m: int, length: int, nstripes: int,
                        strip_stride: int, stripe_stride: int) -> int:
    return lib().orc_simd_encode_strided(k, m, length, nstripes, buf.ctypes.data, strip_stride,
                                         stripe_stride)


def simd_recover_strided(buf: np.ndarray, k: int, m: int, length: int, nstripes: int,
                         strip_stride: int, stripe_stride: int, fail: np.ndarray) -> int:
    fail = np.ascontiguousarray(fail, dtype=np.uint8)
    return lib().orc_simd_recover_strided(k, m, length, nstripes, buf.ctypes.data, strip_stride,
                                          stripe_stride, fail.ctypes.data)


def bench_encode_reconstruct(buf: np.ndarray, k: int, m: int, length: int, nstripes: int,
                             strip_stride: int, stripe_stride: int, fail: np.ndarray,
                             with_reconstruct: bool, nthreads: int, min_seconds: float,
                             simd: bool = False):
    """Times the scalar restatement (simd=False) or the AVX-512 one (simd=True)."""
    passes = C.c_uint64()
    fail = np.ascontiguousarray(fail, dtype=np.uint8)
    el = lib().orc_bench_encode_reconstruct_impl(int(simd), k, m, length, nstripes,
                                                 buf.ctypes.data, strip_stride, stripe_stride,
                                                 fail.ctypes.data, int(with_reconstruct),
                                                 nthreads, min_seconds, C.byref(passes))
    return el, passes.value


def bdevperf_raid5_fsw(n: int = 5, strip: int = 65536, disk_bytes: int = 256 << 20,
                       seconds: float = 10.0, qd: int = 32):
    """BASELINE config 1 CPU harness: (MiB/s, ios, verified)."""
    ios = C.c_uint64()
    ok = C.c_ubyte()
    mibs = lib().orc_bdevperf_raid5_fsw(n, strip, disk_bytes, qd, seconds, C.byref(ios),
                                        C.byref(ok))
    return mibs, ios.value, bool(ok.value)
