"""Runs the C test harness of the host RAID layer (tests/c/test_draid_raid.c):
host logic on CPU, the full-stripe write / degraded read paths on the GPU."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "c", "test_draid_raid")


def _build():
    import draid_ec
    import oracle
    draid_ec.build()
    oracle.build()
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "c")])


def test_c_harness_host_logic():
    _build()
    out = subprocess.run([BIN, "--cpu-only"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "PASS" in out.stdout


def test_per_device_state_keying():
    """State that lives in one GPU's memory is kept per GPU (csrc/per_device.hpp): a
    thread that moves from GPU 0 to GPU 1 never gets GPU 0's scratch, and a device
    address is only vouched for on the GPU that owns it.  Pure host logic, under
    ASan + UBSan."""
    _build()
    out = subprocess.run([os.path.join(HERE, "c", "test_per_device")], capture_output=True,
                         text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "PASS" in out.stdout


@pytest.mark.gpu
def test_c_harness_gpu(ec):
    _build()
    out = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "PASS" in out.stdout


@pytest.mark.gpu
def test_pageable_memory_through_the_c_abi(ec):
    """tests/c/test_pageable.c: malloc'd vectors through the isa-l-shaped calls on both
    sides of the pinned-arena limit, and malloc'd strided stripes (with gaps, partial last
    chunks, mixed failure tables) through draid_ec_host_encode / _reconstruct, bit-exact
    against the oracle."""
    _build()
    out = subprocess.run([os.path.join(HERE, "c", "test_pageable")], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "PASS pageable" in out.stdout


def test_c_sanitizers():
    """The host code under sanitizers.  The host RAID layer and
    stripe cache (compiled from source into the harness) under ASan + UBSan
    and under TSan (the 8-thread stripe-cache test), and the oracle's round
    trips under ASan + UBSan -- host paths only, no GPU."""
    _build()
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "c"), "san"])
    for name, args in (("test_draid_raid_asan", ["--cpu-only"]),
                       ("test_draid_raid_tsan", ["--cpu-only"]),
                       ("test_oracle_san", [])):
        out = subprocess.run([os.path.join(HERE, "c", name)] + args, capture_output=True,
                             text=True, timeout=300)
        if "tsan" in name and "unexpected memory mapping" in out.stderr:
            continue  # TSan cannot start under this kernel's address-space layout
        assert out.returncode == 0, (name, out.stdout[-2000:], out.stderr[-4000:])
        assert "PASS" in out.stdout, name
