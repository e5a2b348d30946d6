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


@pytest.mark.gpu
def test_c_harness_gpu(ec):
    _build()
    out = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "PASS" in out.stdout
