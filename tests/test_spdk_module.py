"""The engine under the reference's own code (binaries under tests/spdk/build/, built by
tests/spdk/Makefile from reference sources where they lie):

* spdk_raid_module_test -- draid-spdk_amd/spdk/raid_gpu.c (a `struct raid_bdev_module`
  for RAID6, and RAID5) linked with the reference's bdev_raid.c: full-stripe, partial and
  degraded I/O through raid_bdev_submit_request, completed from the module's poller, every
  disk byte checked against the oracle, disks failed through base_info->degraded;
* spdk_raid_threads_test -- the same module on four SPDK threads with one channel each:
  requests from all of them interleaved on the same stripes (stepped from one OS thread,
  then with one OS thread per SPDK thread), cross-thread hand-off of a stripe observed, a
  base bdev hot-removed under I/O (the reference's behaviour: the array goes offline);
* spdk_raid_hotremove_test -- the hot-remove with the documented one-statement redirect
  compiled into the reference's framework: the array stays online, degraded;
* spdk_raid5_simple_test -- the reference's raid5_simple.c, unmodified, calling xor_gen at
  its own call site with the engine behind it, on raid5_ut_ref.c's known-answer flow;
* gf_vect_mul_ref -- the reference's P+Q example, unmodified, with its own self-checks.

The binaries hold reference object code, so they are built only where /root/reference
exists (this container) and travel to the GPU box prebuilt.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "spdk", "build")
BINARIES = ("spdk_raid_module_test", "spdk_raid5_simple_test", "gf_vect_mul_ref",
            "spdk_raid_threads_test", "spdk_raid_hotremove_test", "spdk_raid_module_bench")


def build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "draid-spdk_amd"),
                           "libdraid_ec.so", "libdraid_isal.so"])
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"])
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "spdk")])


@pytest.mark.skipif(not os.path.isdir(REF), reason="needs the reference tree to compile against")
def test_module_compiles_against_the_reference_headers_and_links_with_its_framework():
    build()
    for b in BINARIES:
        assert os.access(os.path.join(OUT, b), os.X_OK), b
    # the module registers through the reference's RAID_MODULE_REGISTER, and the binary
    # carries the reference's framework, not a restatement of it
    syms = subprocess.run(["nm", os.path.join(OUT, "spdk_raid_module_test")], capture_output=True,
                          text=True, check=True).stdout
    for name in ("raid_bdev_module_list_add", "raid_bdev_create", "raid_bdev_add_base_devices",
                 "raid_bdev_io_complete", "raid_gpu_set_degraded", "g_raid_bdev_list"):
        assert f" {name}" in syms, name
    undefined = subprocess.run(["nm", "-u", os.path.join(OUT, "raid_gpu.o")], capture_output=True,
                               text=True, check=True).stdout
    # the module's parity arithmetic is the C ABI, nothing else
    assert "draid_ec_ctx_flush_ticket" in undefined and "draid_raid_stripe_write" in undefined
    assert "orc_" not in undefined and "xor_gen" not in undefined
    # the redirect is in the second framework object and only there
    for obj, want in (("bdev_raid_ref.o", False), ("bdev_raid_hotremove.o", True)):
        u = subprocess.run(["nm", "-u", os.path.join(OUT, obj)], capture_output=True, text=True,
                           check=True).stdout
        assert ("raid_gpu_base_bdev_removed" in u) == want, obj
    # the shim exports isa-l's names
    shim = subprocess.run(["nm", "-D", os.path.join(ROOT, "draid-spdk_amd", "libdraid_isal.so")],
                          capture_output=True, text=True, check=True).stdout
    for name in ("xor_gen", "pq_gen", "pq_check_base", "gf_vect_mul", "gf_vect_mul_init", "gf_mul",
                 "gf_inv"):
        assert f" T {name}\n" in shim, name


def run(binary, timeout=300, env=None):
    path = os.path.join(OUT, binary)
    if not os.access(path, os.X_OK):
        pytest.fail(f"{path} is missing: build it with `make -C tests/spdk` where the reference "
                    "tree is available (it ships to the GPU box prebuilt)")
    p = subprocess.run([path], capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, **(env or {})))
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return p.stdout


@pytest.mark.gpu
def test_raid6_module_under_the_reference_framework():
    out = run("spdk_raid_module_test")
    assert "ok raid6 n=10 strip=64KiB" in out and "ok raid5 n=5 strip=64KiB" in out
    assert "array checks passed" in out


@pytest.mark.gpu
def test_raid6_module_routes_stripes_over_several_device_slots():
    """DRAID_RAID_GPUS=3 on a box with fewer GPUs puts several slots on one device:
    one context per slot and channel, stripe s on slot s mod 3, every slot flushed and
    polled by the channel's poller.  The same array checks must pass."""
    out = run("spdk_raid_module_test", env={"DRAID_RAID_GPUS": "3"})
    assert "ok raid6 n=10 strip=64KiB" in out and "array checks passed" in out


@pytest.mark.gpu
def test_raid6_module_with_a_request_pool_of_four():
    """DRAID_RAID_REQUESTS=4: parent I/O beyond the channel's four stripe requests waits on
    the channel's retry list and is resubmitted, in submission order, as requests complete
    (raid5_simple.c:364-370); the same array checks must pass.  (One channel: with several,
    I/O that waits takes its place in a stripe's queue only when it gets a request, so
    requests of different channels to one stripe may then run out of submission order --
    as in the reference, which completes such I/O with NOMEM for the bdev layer to retry,
    raid5.c:993-997.)"""
    out = run("spdk_raid_module_test", env={"DRAID_RAID_REQUESTS": "4"})
    assert "ok raid6 n=10 strip=64KiB" in out and "array checks passed" in out
    # 32 requests outstanding over a pool of eight: 24 always wait, all complete, none fails
    import json
    p = subprocess.run([os.path.join(OUT, "spdk_raid_module_bench"), "6", "10", "64", "32", "0.3"],
                       capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, DRAID_RAID_REQUESTS="8"))
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    rows = [json.loads(line) for line in p.stdout.splitlines() if line.startswith("{")]
    assert len(rows) == 5 and all(r["failed"] == 0 and r["ios"] > 100 for r in rows)
    # waiting I/O is served in submission order: no task is left behind while the others
    # resubmit from their completion callbacks
    for r in rows:
        assert r["task_ios_min"] * 2 >= r["task_ios_max"] > 0, r


@pytest.mark.gpu
def test_module_on_four_spdk_threads_and_through_hot_remove():
    """raid5.c:496-505,1047-1054: requests of one stripe run one at a time, in arrival
    order, and a finished request hands the stripe to the next one's thread.  Four channels
    on four SPDK threads hit the same stripes; every read must see the writes submitted
    before it, every disk byte must match the oracle, and at least one hand-off must cross
    threads.  Then a base bdev is removed under I/O (bdev_raid.c:1333-1390)."""
    out = run("spdk_raid_threads_test")
    assert "ok interleaved: 4 SPDK threads" in out
    assert out.count("ok OS threads: 4 pthreads") == 2
    assert "ok hot-remove, reference behaviour: array offline" in out
    hand = [ln for ln in out.splitlines() if "interleaved:" in ln and "hand-offs" in ln]
    assert hand and int(hand[0].split("hand-offs")[1].split(",")[0]) > 0, hand


@pytest.mark.gpu
def test_module_on_four_spdk_threads_over_several_device_slots():
    """The same four-thread run with three device slots per channel (DRAID_RAID_GPUS=3, all
    on the one GPU): every channel owns three contexts, a stripe's slot is s mod 3 whatever
    thread its request came from, and each slot has its own launches in flight."""
    out = run("spdk_raid_threads_test", env={"DRAID_RAID_GPUS": "3"})
    assert "ok interleaved: 4 SPDK threads" in out
    assert out.count("ok OS threads: 4 pthreads") == 2
    assert "ok hot-remove, reference behaviour: array offline" in out


@pytest.mark.gpu
def test_hot_remove_with_the_redirect_keeps_the_array_online():
    out = run("spdk_raid_hotremove_test")
    assert "ok hot-remove with the redirect: online through two removals, offline at the third" in out


@pytest.mark.gpu
def test_module_sustains_queue_depth_32():
    """The bdevperf-shaped harness (full-stripe writes, strip writes, healthy and degraded
    reads with 32 requests outstanding on one reactor): every request completes, none fails,
    and the poller batches several requests into each launch."""
    import json
    path = os.path.join(OUT, "spdk_raid_module_bench")
    if not os.access(path, os.X_OK):
        pytest.fail(f"{path} is missing: build it with `make -C tests/spdk`")
    p = subprocess.run([path, "6", "10", "64", "32", "0.3"], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    rows = [json.loads(line) for line in p.stdout.splitlines() if line.startswith("{")]
    assert [r["job"] for r in rows] == ["full_stripe_write", "strip_write_rmw", "full_stripe_read",
                                        "full_stripe_read_1_degraded", "full_stripe_read_2_degraded"]
    assert all(r["failed"] == 0 and r["ios"] > 100 for r in rows)
    assert rows[0]["requests_per_launch"] > 2 and rows[4]["launches"] > 0


@pytest.mark.gpu
def test_reference_raid5_simple_calls_the_engine_at_its_xor_gen_call_site():
    out = run("spdk_raid5_simple_test")
    assert "stripe parities equal the known answer" in out


@pytest.mark.gpu
def test_reference_pq_example_passes_unmodified_on_the_engine():
    out = run("gf_vect_mul_ref")
    assert "done: Pass" in out
