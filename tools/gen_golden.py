#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (committed with this script).

Sources of truth, in order of strength:

1. ``gf_vect_mul.c`` scenarios (examples/bdev/gf_vect_mul/gf_vect_mul.c:68-347):
   glibc ``srand(0x1234)`` + ``rand()`` inputs drawn in the example's exact call
   order (rand test :142-144, block test :189-191, D+P :243-245, D+D :284-286),
   k = 14, len = 4096.  We store P||Q of each scenario plus SHA-256 of the inputs;
   the example's own self-checks are re-run in tests/test_oracle.py.
2. ``raid5_ut_ref.c`` XOR known-answer (test/unit/lib/bdev/raid/raid5.c/
   raid5_ut_ref.c:324-330,350-397): 0xFF fill + 8-byte LE block index per block,
   parity = XOR of the k data strips, for n in {3,4,5}, blocklen in {512,4096},
   strip in {1,4} KiB (strip_size = 0 cases skipped as raid5_ut.c:96-100 does).
3. splitmix64-seeded stripes (4+1, 8+2, 16+2 at 4 KiB full bytes; config sizes as
   SHA-256 manifests), with every recoverable failure set's output hashed.
4. GF(2^8) exp / log / inverse tables (poly 0x11D, generator 2).

Everything is computed by the C oracle and cross-checked against the
independent numpy restatement before being written.
"""
from __future__ import annotations

import hashlib
import itertools
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from oracle import np_ref  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def sha(b: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(b).tobytes()).hexdigest()


def stripe_seed(s: int, j: int) -> int:
    """Seed of strip j of stripe s (a fixed function of s and j, so the fixture can be regenerated)."""
    return (0x1234 ^ (s << 16) ^ j) & 0xFFFFFFFFFFFFFFFF


def splitmix_stripe(k: int, m: int, length: int, s: int) -> list[np.ndarray]:
    return [oracle.fill_splitmix(length, stripe_seed(s, j)) for j in range(k)] + \
           [np.zeros(length, np.uint8) for _ in range(m)]


def gf_vect_mul_scenarios(man: dict) -> None:
    K, L = 14, 4096
    oracle.srand(0x1234)
    names = ["rand", "blocks", "d_plus_p", "d_plus_d"]
    scen = {}
    for name in names:
        data = [oracle.rand_buffer(L) for _ in range(K)]
        vec = data + [np.zeros(L, np.uint8), np.zeros(L, np.uint8)]
        assert oracle.pq_gen(vec, L) == 0
        p, q = np_ref.pq_gen(np.stack(data))
        assert (vec[K] == p).all() and (vec[K + 1] == q).all()
        pq = np.concatenate([vec[K], vec[K + 1]])
        fn = f"gfvm_{name}_pq.bin"
        pq.tofile(os.path.join(OUT, fn))
        scen[name] = {"inputs_sha256": sha(np.stack(data)), "pq_file": fn,
                      "pq_sha256": sha(pq)}
    man["gf_vect_mul_example"] = {"k": K, "len": L, "seed": 0x1234, "scenarios": scen,
                                  "order": names}


def ut_ref_xor(man: dict) -> None:
    cases = []
    for n in (3, 4, 5):
        for blocklen in (512, 4096):
            for strip_kb in (1, 4):
                strip = strip_kb * 1024 // blocklen
                if strip == 0:
                    continue
                k = n - 1
                stripe_blocks = strip * k
                buf = oracle.ut_ref_pattern(stripe_blocks, blocklen)
                S = strip * blocklen
                data = [buf[j * S:(j + 1) * S].copy() for j in range(k)]
                par = np.zeros(S, np.uint8)
                assert oracle.xor_gen(data + [par], S) == 0
                assert (par == np_ref.xor_gen(np.stack(data))).all()
                fn = f"ut_ref_n{n}_bl{blocklen}_s{strip_kb}k_parity.bin"
                par.tofile(os.path.join(OUT, fn))
                cases.append({"n": n, "blocklen": blocklen, "strip_kb": strip_kb,
                              "parity_file": fn, "parity_sha256": sha(par)})
    man["raid5_ut_ref"] = cases


def splitmix_cases(man: dict) -> None:
    full = []
    for k, m in ((4, 1), (8, 2), (16, 2)):
        L = 4096
        for s in (0, 1):
            strips = splitmix_stripe(k, m, L, s)
            rc = oracle.xor_gen(strips, L) if m == 1 else oracle.pq_gen(strips, L)
            assert rc == 0
            ref = np.stack(strips)
            if m == 1:
                assert (ref[k] == np_ref.xor_gen(ref[:k])).all()
            else:
                p, q = np_ref.pq_gen(ref[:k])
                assert (ref[k] == p).all() and (ref[k + 1] == q).all()
            fn = f"splitmix_k{k}_m{m}_s{s}_parity.bin"
            ref[k:].tofile(os.path.join(OUT, fn))
            rec = {}
            for nf in range(1, m + 1):
                for fail in itertools.combinations(range(k + m), nf):
                    v = [x.copy() for x in strips]
                    for f in fail:
                        v[f][:] = 0
                    assert oracle.recover(v, k, m, L, list(fail)) == 0
                    assert all((v[j] == ref[j]).all() for j in range(k + m))
            rec["all_single_and_double_failures"] = "round-trip to the encoded stripe"
            full.append({"k": k, "m": m, "len": L, "stripe": s, "parity_file": fn,
                         "parity_sha256": sha(ref[k:]), "data_sha256": sha(ref[:k]),
                         "recover": rec})
    man["splitmix_4k"] = full

    cfg = []
    for k, m, L, ns in ((4, 1, 65536, 4), (8, 2, 65536, 4), (8, 2, 131072, 2), (16, 2, 262144, 2)):
        ent = {"k": k, "m": m, "len": L, "stripes": []}
        for s in range(ns):
            strips = splitmix_stripe(k, m, L, s)
            rc = oracle.xor_gen(strips, L) if m == 1 else oracle.pq_gen(strips, L)
            assert rc == 0
            ent["stripes"].append({"stripe": s, "data_sha256": sha(np.stack(strips[:k])),
                                   "parity_sha256": sha(np.stack(strips[k:]))})
        cfg.append(ent)
    man["splitmix_config_sizes"] = cfg


def gf_tables(man: dict) -> None:
    e, g = oracle.gf_tables()
    inv = np.array([oracle.gf_inv(a) for a in range(256)], np.uint8)
    assert (inv == np_ref.INV).all()
    tab = np.concatenate([e, g, inv])
    tab.tofile(os.path.join(OUT, "gf_exp_log_inv.bin"))
    man["gf_tables"] = {"file": "gf_exp_log_inv.bin", "layout": "exp[256] log[256] inv[256]",
                        "sha256": sha(tab),
                        "spot": {"gf_mul(0x80,2)": oracle.gf_mul(0x80, 2),
                                 "gf_inv(2)": oracle.gf_inv(2),
                                 "2^8": oracle.gf_pow2(8), "2^254": oracle.gf_pow2(254)}}


def main() -> None:
    os.makedirs(OUT, exist_ok=True)
    man: dict = {"generator": "tools/gen_golden.py", "field": {"poly": 0x11D, "generator": 2},
                 "stripe_seed": "splitmix64 state = 0x1234 ^ (stripe << 16) ^ strip"}
    gf_tables(man)
    gf_vect_mul_scenarios(man)
    ut_ref_xor(man)
    splitmix_cases(man)
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
