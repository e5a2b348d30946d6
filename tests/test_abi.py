"""CPU tests of the C ABI: libdraid_ec.so loads, exports every symbol the header
declares, and the host-side scalar GF helpers agree with the oracle.  No compute
call is made (there is no GPU here)."""
import ctypes
import os
import re
import shutil
import subprocess

import oracle

import draid_ec


INCLUDE = os.path.dirname(draid_ec.HEADER)


def header_functions(path):
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(draid_\w+)\s*\(", txt)))


def test_library_exports_header_symbols():
    draid_ec.build()
    L = ctypes.CDLL(draid_ec.LIB_PATH)
    headers = [os.path.join(INCLUDE, f) for f in sorted(os.listdir(INCLUDE)) if f.endswith(".h")]
    assert len(headers) >= 2
    total = 0
    for h in headers:
        for n in header_functions(h):
            assert hasattr(L, n), f"libdraid_ec.so does not export {n} ({h})"
            total += 1
    assert total >= 35
    # the ctypes binding declares exactly the C ABI of draid_ec.h
    assert sorted(draid_ec.EXPORTS) == header_functions(draid_ec.HEADER)


def test_library_is_gfx950_code_object(tmp_path):
    # --offloading extracts the bundles next to its input: run it on a copy
    lib = tmp_path / "libdraid_ec.so"
    shutil.copy(draid_ec.LIB_PATH, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", "-h", str(lib)],
                         capture_output=True, text=True, cwd=str(tmp_path))
    blob = out.stdout + out.stderr
    if "gfx" not in blob:  # older objdump: fall back to strings in the bundle
        blob = open(draid_ec.LIB_PATH, "rb").read().decode("latin-1")
    assert "gfx950" in blob


def test_no_oracle_in_product():
    """The product library must not link or reference the CPU oracle."""
    data = open(draid_ec.LIB_PATH, "rb").read()
    assert b"liboracle" not in data and b"orc_" not in data
    csrc = os.path.join(os.path.dirname(draid_ec.LIB_PATH), "csrc")
    for f in os.listdir(csrc):
        assert "oracle" not in open(os.path.join(csrc, f)).read()


def test_abi_version_and_host_gf():
    assert draid_ec.lib().draid_ec_abi_version() == 1
    for a in range(256):
        assert draid_ec.gf_inv(a) == oracle.gf_inv(a)
        for b in range(0, 256, 5):
            assert draid_ec.gf_mul(a, b) == oracle.gf_mul(a, b)
    for c in (0, 1, 2, 0x1D, 0x8E, 0xFF):
        assert draid_ec.gf_vect_mul_init(c) == bytes(oracle.gf_vect_mul_init(c))


def test_argument_errors_before_any_launch():
    """Rejected arguments return 1 (isa-l style) before any HIP call, so this runs
    without a GPU: bad k/m/flags, NULL tables, and launches too large for one grid."""
    import ctypes as C
    L = draid_ec.lib()
    dummy = C.c_void_p(0x1000)
    cases = [
        draid_ec.StripeBatch(0, 2, 4096, 1, 0, dummy.value),        # k = 0
        draid_ec.StripeBatch(8, 3, 4096, 1, 0, dummy.value),        # m = 3
        draid_ec.StripeBatch(8, 2, 4096, 1, 7, dummy.value),        # flags != 0
        draid_ec.StripeBatch(8, 2, 4096, 1, 0, None),               # no table
        draid_ec.StripeBatch(8, 2, 0x80000000, 1, 0, dummy.value),  # strip > 0x7fff0000
        draid_ec.StripeBatch(8, 2, 1 << 30, 4096, 0, dummy.value),  # 2^32 work items
    ]
    for b in cases:
        assert L.draid_ec_encode(C.byref(b), None) == 1, draid_ec.last_error()
    assert L.draid_ec_reconstruct(C.byref(cases[-1]), dummy, None) == 1
    assert "too large" in draid_ec.last_error()
    # failure indices are bytes with 0xFF = none: reconstructs need k + m <= 255
    wide = draid_ec.StripeBatch(254, 2, 4096, 1, 0, dummy.value)
    assert L.draid_ec_reconstruct(C.byref(wide), dummy, None) == 1
    assert "k + m <= 255" in draid_ec.last_error()
    arr257 = (C.c_void_p * 257)(*([dummy.value] * 257))
    f = (C.c_int * 1)(0)
    assert L.draid_recover(255, 2, 64, arr257, 1, f) == 1
    h = draid_ec.HostStripes(8, 2, 1 << 30, 4096, 0, dummy.value, 1 << 30, 10 << 30)
    assert L.draid_ec_encode_strided(C.byref(h), None) == 1
    assert L.draid_ec_host_encode(C.byref(h), 0) == 1
    # isa-l contracts of the synchronous calls
    arr = (C.c_void_p * 4)(*([dummy.value] * 4))
    assert L.draid_xor_gen(2, 64, arr) == 1           # fewer than 2 sources + dest
    assert L.draid_pq_gen(4, 48, arr) == 1            # len % 32 != 0
    assert L.draid_gf_vect_mul(31, bytes(32), dummy, dummy) == 1
    # NULL out-pointers of the runtime helpers
    assert L.draid_ec_device_count(None) == 1
    assert L.draid_ec_stream_create(None) == 1
    assert L.draid_ec_device_alloc(None, C.c_size_t(64)) == 1
    assert L.draid_ec_host_device_pointer(dummy, None) == 1
    assert L.draid_ec_ctx_set_autoflush(None, C.c_uint64(1024)) == 1


def test_every_registered_kernel_has_device_code():
    """The host half of the library registers its kernels by mangled name and the GPU half
    must hold a kernel descriptor (`<name>.kd`) for each: hipcc compiles the two halves in
    separate passes over the source, and a library whose halves disagree (a source edited
    while it was being compiled) aborts the process at the first launch."""
    import subprocess
    import draid_ec
    out = subprocess.run(["strings", "-a", draid_ec.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout.splitlines()
    device = {s[:-3] for s in out if s.endswith(".kd")}
    # what the host registers: the kernels' mangled names as plain strings (the stubs
    # and the descriptors' own attributes carry other spellings)
    registered = {s for s in out if s.startswith("_ZN5draid") and "__device_stub__" not in s
                  and "." not in s and s.split("I")[0].split("E")[0][len("_ZN5draid"):].lstrip(
                      "0123456789").startswith("k_")}
    assert len(device) > 200 and len(registered) > 200
    missing = registered - device
    assert not missing, sorted(missing)[:3]
    assert device <= registered | device and len(registered & device) == len(registered)
