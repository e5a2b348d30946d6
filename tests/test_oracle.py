"""CPU tests: pin the oracle against the reference's own test material.

* gf_vect_mul.c's five scenarios (examples/bdev/gf_vect_mul/gf_vect_mul.c:95-347)
  re-run step by step on glibc srand(0x1234)/rand() inputs, plus the committed
  P||Q fixtures.
* raid5_ut_ref.c's XOR known answer (test/unit/lib/bdev/raid/raid5.c/
  raid5_ut_ref.c:324-330,350-397).
* raid5_ut.c's geometry grid (test/unit/lib/bdev/raid/raid5.c/raid5_ut.c:61-105,176-195).
* An independent numpy restatement (oracle/np_ref.py) on random stripes.
"""
import hashlib
import itertools
import os

import numpy as np
import pytest

import oracle
from oracle import np_ref


def sha(b):
    return hashlib.sha256(np.ascontiguousarray(b).tobytes()).hexdigest()


def test_gf_field_spot_values(golden):
    assert oracle.gf_mul(0x80, 2) == 0x1D
    assert oracle.gf_inv(2) == 0x8E
    assert oracle.gf_pow2(8) == 0x1D
    assert oracle.gf_pow2(255) == 1
    for a in range(1, 256):
        assert oracle.gf_mul(a, oracle.gf_inv(a)) == 1
    tab = np.fromfile(os.path.join(golden["_dir"], golden["gf_tables"]["file"]), np.uint8)
    assert sha(tab) == golden["gf_tables"]["sha256"]
    e, g = oracle.gf_tables()
    assert (tab[:256] == e).all() and (tab[256:512] == g).all()


def test_gf_mul_matches_independent_table():
    for a in range(256):
        for b in range(0, 256, 7):
            assert oracle.gf_mul(a, b) == np_ref.gf_mul(a, b)
    for c in range(256):
        assert (oracle.gf_vect_mul_init(c) == np_ref.gf_vect_mul_init(c)).all()


def _gfvm_tables():
    """gf_const_tbl_arr[i] = gf_vect_mul_init(2^i) built by repeated gf_mul(c, 2)."""
    tbls = []
    for i in range(255):
        c = 1
        for _ in range(i):
            c = oracle.gf_mul(c, 2)
        tbls.append(oracle.gf_vect_mul_init(c))
    return tbls


def test_gf_vect_mul_example_scenarios(golden):
    """Replays gf_vect_mul.c's main() on the oracle (same call order, same seed)."""
    K, L = 14, 4096
    tb = _gfvm_tables()
    z = lambda: np.zeros(L, np.uint8)  # noqa: E731
    gm = golden["gf_vect_mul_example"]

    # zero test :95-139
    buffs = [z() for _ in range(K + 2)]
    assert oracle.pq_gen(buffs, L) == 0
    assert not buffs[K].any() and not buffs[K + 1].any()

    oracle.srand(0x1234)
    # random test :141-186
    for name in gm["order"]:
        buffs = [oracle.rand_buffer(L) for _ in range(K)] + [z(), z()]
        assert sha(np.stack(buffs[:K])) == gm["scenarios"][name]["inputs_sha256"]
        assert oracle.pq_gen(buffs, L) == 0
        pq = np.fromfile(os.path.join(golden["_dir"], gm["scenarios"][name]["pq_file"]), np.uint8)
        assert (np.concatenate([buffs[K], buffs[K + 1]]) == pq).all()
        b2 = [z() for _ in range(K + 2)]
        if name in ("rand", "blocks"):
            step = L if name == "rand" else 512
            for i in range(K):
                for j in range(0, L, step):
                    assert oracle.xor_gen([buffs[i][j:j + step], b2[K][j:j + step],
                                           b2[K][j:j + step]], step) == 0
                    assert oracle.gf_vect_mul(step, tb[i], buffs[i][j:j + step],
                                              b2[i][j:j + step]) == 0
            for i in range(K):
                for j in range(0, L, step):
                    assert oracle.xor_gen([b2[i][j:j + step], b2[K + 1][j:j + step],
                                           b2[K + 1][j:j + step]], step) == 0
            for i in range(K):
                b2[i][:] = buffs[i]
            assert oracle.pq_check(buffs, L) == 0
            assert oracle.pq_check(b2, L) == 0
        elif name == "d_plus_p":  # :242-281
            for i in range(K):
                oracle.gf_vect_mul(L, tb[i], buffs[i], b2[i])
            for i in range(K):
                if i != 3:
                    oracle.xor_gen([b2[i], b2[K + 1], b2[K + 1]], L)
            oracle.xor_gen([buffs[K + 1], b2[K + 1], b2[K + 1]], L)
            oracle.gf_vect_mul(L, tb[255 - 3], b2[K + 1], b2[3])
            assert (b2[3] == buffs[3]).all()
        else:  # d_plus_d :283-347
            for i in range(K):
                oracle.gf_vect_mul(L, tb[i], buffs[i], b2[i])
            for i in range(K):
                if i in (3, 8):
                    continue
                oracle.xor_gen([buffs[i], b2[K], b2[K]], L)
                oracle.xor_gen([b2[i], b2[K + 1], b2[K + 1]], L)
            oracle.xor_gen([buffs[K], b2[K], b2[K]], L)
            oracle.xor_gen([buffs[K + 1], b2[K + 1], b2[K + 1]], L)
            gyx, gmx = 1, 1
            for _ in range(8 - 3):
                gyx = oracle.gf_mul(gyx, 2)
            for _ in range(255 - 3):
                gmx = oracle.gf_mul(gmx, 2)
            a = oracle.gf_mul(gyx, oracle.gf_inv(gyx ^ 1))
            b = oracle.gf_mul(gmx, oracle.gf_inv(gyx ^ 1))
            tmp = z()
            oracle.gf_vect_mul(L, oracle.gf_vect_mul_init(a), b2[K], tmp)
            oracle.gf_vect_mul(L, oracle.gf_vect_mul_init(b), b2[K + 1], b2[3])
            oracle.xor_gen([tmp, b2[3], b2[3]], L)
            b2[8][:] = b2[3]
            oracle.xor_gen([b2[K], b2[8], b2[8]], L)
            assert (b2[3] == buffs[3]).all() and (b2[8] == buffs[8]).all()
        # the oracle's composite recovery reproduces the same strips
        for fail in ([3, K], [3, 8], [3], [K, K + 1], [5, K + 1]):
            v = [x.copy() for x in buffs]
            for f in fail:
                v[f][:] = 0x5A
            assert oracle.recover(v, K, 2, L, fail) == 0
            assert all((v[j] == buffs[j]).all() for j in range(K + 2))


@pytest.mark.parametrize("case", range(9))
def test_raid5_ut_ref_known_answer(golden, case):
    c = golden["raid5_ut_ref"][case]
    n, bl, skb = c["n"], c["blocklen"], c["strip_kb"]
    strip = skb * 1024 // bl
    k = n - 1
    buf = oracle.ut_ref_pattern(strip * k, bl)
    S = strip * bl
    ref = np.zeros(S, np.uint8)
    for j in range(k):  # raid5_ut_ref.c:324-330 xor_block
        ref ^= buf[j * S:(j + 1) * S]
    par = np.zeros(S, np.uint8)
    assert oracle.xor_gen([buf[j * S:(j + 1) * S] for j in range(k)] + [par], S) == 0
    assert (par == ref).all()
    assert (par == np.fromfile(os.path.join(golden["_dir"], c["parity_file"]), np.uint8)).all()


def test_private_rand_state_matches_glibc_rand():
    """orc_srand/orc_rand_buffer (random_r, private state) == srand/rand."""
    oracle.glibc_srand(0x1234)
    a = oracle.glibc_rand_buffer(3 * 4096)
    oracle.srand(0x1234)
    b = oracle.rand_buffer(3 * 4096)
    assert (a == b).all()


def test_raid5_geometry_grid():
    """raid5_ut.c:61-105 parameter grid and :176-195 assertions."""
    for n in (3, 4, 5):
        for blockcnt in (1, 1024, 1024 * 1024):
            for bl in (512, 4096):
                for skb in (1, 4, 128):
                    strip = skb * 1024 // bl
                    if strip == 0 or strip > blockcnt:
                        continue
                    sb, ts, bc, oib = oracle.raid5_start_geometry(n, 1, blockcnt, strip)
                    assert sb == strip * (n - 1)
                    assert ts == blockcnt // strip
                    assert bc == (blockcnt - blockcnt % strip) * (n - 1)
                    assert oib == sb
    # parity rotation raid5.c:1006-1007: p = (n-1) - s mod n
    assert [oracle.raid5_parity_chunk(5, 1, s) for s in range(6)] == [4, 3, 2, 1, 0, 4]
    assert [oracle.raid5_data_chunk_to_disk(2, d) for d in range(4)] == [0, 1, 3, 4]


@pytest.mark.parametrize("k,m", [(2, 1), (4, 1), (8, 2), (16, 2), (14, 2), (3, 2)])
def test_oracle_vs_numpy_all_failures(k, m):
    rng = np.random.default_rng(k * 10 + m)
    L = 1024
    d = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    par = [np.zeros(L, np.uint8) for _ in range(m)]
    rc = oracle.xor_gen(d + par, L) if m == 1 else oracle.pq_gen(d + par, L)
    assert rc == 0
    p, q = np_ref.pq_gen(np.stack(d))
    assert (par[0] == p).all()
    if m == 2:
        assert (par[1] == q).all()
    strips = np.stack(d + par)
    for nf in range(1, m + 1):
        for fail in itertools.combinations(range(k + m), nf):
            v = [s.copy() for s in strips]
            for f in fail:
                v[f][:] = 0xA5
            assert oracle.recover(v, k, m, L, list(fail)) == 0
            assert all((v[j] == strips[j]).all() for j in range(k + m)), fail
            assert (np_ref.recover(np.stack(v), k, m, list(fail)) == strips).all()


@pytest.mark.parametrize("m", [1, 2])
def test_oracle_single_data_strip(m):
    """k = 1 (the GPU batch API accepts it): every parity strip is a copy of D0
    and each single / dual failure set rebuilds."""
    L, B = 1000, 3
    rng = np.random.default_rng(m)
    buf = np.zeros((B, 1 + m, L), np.uint8)
    buf[:, 0] = rng.integers(0, 256, (B, L), dtype=np.uint8)
    assert oracle.encode_strided(buf.reshape(-1), 1, m, L, B, L, (1 + m) * L) == 0
    for j in range(1, 1 + m):
        assert (buf[:, j] == buf[:, 0]).all()
    good = buf.copy()
    sets = [(0, 0xFF), (1, 0xFF)] + ([(0, 1), (2, 0), (1, 2)] if m == 2 else [])
    for f in sets:
        fail = np.tile(np.array(f, np.uint8), B)
        for j in f:
            if j != 0xFF:
                buf[:, j] = 0x5A
        assert oracle.recover_strided(buf.reshape(-1), 1, m, L, B, L, (1 + m) * L, fail) == 0
        assert (buf == good).all(), f


def test_splitmix_fixtures(golden):
    from tools.gen_golden import splitmix_stripe
    for c in golden["splitmix_4k"]:
        k, m, L = c["k"], c["m"], c["len"]
        strips = splitmix_stripe(k, m, L, c["stripe"])
        rc = oracle.xor_gen(strips, L) if m == 1 else oracle.pq_gen(strips, L)
        assert rc == 0
        par = np.fromfile(os.path.join(golden["_dir"], c["parity_file"]), np.uint8).reshape(m, L)
        assert (np.stack(strips[k:]) == par).all()
        assert sha(np.stack(strips[:k])) == c["data_sha256"]


def test_isal_argument_semantics():
    L = 64
    v = [np.zeros(L, np.uint8) for _ in range(4)]
    assert oracle.xor_gen(v[:2], L) == 1          # fewer than two sources
    assert oracle.xor_gen(v[:3], 17) == 0         # any length
    assert oracle.pq_gen(v[:3], L) == 1           # fewer than two sources
    assert oracle.pq_gen(v, 48) == 1              # len % 32 != 0
    assert oracle.pq_gen(v, 0) == 0
    assert oracle.gf_vect_mul(40, oracle.gf_vect_mul_init(3), v[0], v[1]) == 1
    assert oracle.recover(v, 2, 2, L, [0, 0]) == -1
    assert oracle.recover(v, 2, 1, L, [0, 1]) == -1


def test_bench_sample_runs():
    """The cpu_baseline leg's C timing loop works on a tiny batch."""
    k, m, L, B = 8, 2, 4096, 8
    buf = np.frombuffer(np.random.default_rng(0).bytes((k + m) * L * B), np.uint8).copy()
    fail = np.full(2 * B, 0xFF, np.uint8)
    fail[0::2] = 1
    fail[1::2] = 6
    el, passes = oracle.bench_encode_reconstruct(buf, k, m, L, B, L, (k + m) * L, fail, True, 2, 0.01)
    assert el > 0 and passes >= 1


@pytest.mark.skipif(not oracle.simd_available(), reason="CPU lacks AVX-512BW/GFNI")
@pytest.mark.parametrize("k,m,L", [(1, 2, 200), (2, 1, 64), (4, 1, 4096 + 7), (8, 2, 65536),
                                   (14, 2, 4096), (16, 2, 1000), (3, 2, 129)])
def test_simd_matches_scalar(k, m, L):
    """The AVX-512 restatement (the bench's CPU baseline) is byte-exact with the
    scalar oracle for encode and for every single/double failure set."""
    n = k + m
    pairs = [(x, 0xFF) for x in range(n)]
    if m == 2:
        pairs += [(x, y) for x in range(n) for y in range(n) if x != y]
    B = len(pairs)
    rng = np.random.default_rng(k * 100 + L)
    buf = np.zeros((B, n, L), np.uint8)
    buf[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    ref = buf.copy()
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, n * L) == 0
    got = buf.copy()
    assert oracle.simd_encode_strided(got.reshape(-1), k, m, L, B, L, n * L) == 0
    assert (got == ref).all()
    fail = np.array(pairs, np.uint8)
    for s, (x, y) in enumerate(pairs):
        got[s, x] = 0x5A
        if y != 0xFF:
            got[s, y] = 0xA5
    assert oracle.simd_recover_strided(got.reshape(-1), k, m, L, B, L, n * L,
                                       fail.reshape(-1)) == 0
    assert (got == ref).all()


@pytest.mark.skipif(not oracle.simd_available(), reason="CPU lacks AVX-512BW/GFNI")
@pytest.mark.parametrize("vects,L", [(3, 64), (5, 65536), (3, 1), (17, 4096 + 33)])
def test_simd_xor_gen_matches_scalar(vects, L):
    rng = np.random.default_rng(vects + L)
    a = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(vects - 1)] + [np.zeros(L, np.uint8)]
    b = [x.copy() for x in a]
    assert oracle.xor_gen(a, L) == 0
    assert oracle.simd_xor_gen(b, L) == 0
    assert all((x == y).all() for x, y in zip(a, b))
