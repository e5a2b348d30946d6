"""Which kinds of host memory does hipHostRegister accept on this box?
Prints one line per kind (shared/private anonymous mmap, malloc'd, touched or not)."""
import ctypes, mmap, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "draid-spdk_amd"))
import draid_ec as ec

L = ec.lib()
libc = ctypes.CDLL(None)
libc.mmap.restype = ctypes.c_void_p
libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
libc.posix_memalign.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_size_t]
N = 69632
PROT_RW, MAP_SHARED, MAP_PRIVATE, MAP_ANON = 3, 1, 2, 0x20


def try_reg(name, addr, n, touch):
    if touch:
        ctypes.memset(addr, 1, n)
    rc = L.draid_ec_host_register(ctypes.c_void_p(addr), ctypes.c_size_t(n))
    msg = "" if rc == 0 else ec.last_error()
    print(f"{name:40s} touch={touch} addr={addr:#x} rc={rc} {msg}", flush=True)
    if rc == 0:
        L.draid_ec_host_unregister(ctypes.c_void_p(addr))


import torch
torch.cuda.init()
for touch in (False, True):
    a = libc.mmap(None, N, PROT_RW, MAP_SHARED | MAP_ANON, -1, 0)
    try_reg("mmap shared anonymous", a, N, touch)
    a = libc.mmap(None, N, PROT_RW, MAP_PRIVATE | MAP_ANON, -1, 0)
    try_reg("mmap private anonymous", a, N, touch)
    p = ctypes.c_void_p()
    libc.posix_memalign(ctypes.byref(p), 4096, N)
    try_reg("posix_memalign 4096", p.value, N, touch)
    mm = mmap.mmap(-1, N)
    try_reg("python mmap(-1)", ctypes.addressof(ctypes.c_char.from_buffer(mm)), N, touch)
    a = libc.mmap(None, 4 << 20, PROT_RW, MAP_PRIVATE | MAP_ANON, -1, 0)
    try_reg("mmap private anonymous 4 MiB", a, 4 << 20, touch)
    a = libc.mmap(None, 4 << 20, PROT_RW, MAP_SHARED | MAP_ANON, -1, 0)
    try_reg("mmap shared anonymous 4 MiB", a, 4 << 20, touch)
