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
