#!/usr/bin/env python3
"""Regenerate tests/golden/ from the compiled reference (survey container only).

Builds oracle/_ref/librs_ref.so + gen_golden from /root/reference (oracle/Makefile, sources are
compiled where they lie), runs every case below through the reference's public API
(rs_generate_repair_symbols / rs_restore_symbols) and stores the outputs:
  * outputs <= 256 KiB  -> tests/golden/<name>.bin (raw bytes)
  * larger outputs      -> sha256 only
plus tests/golden/manifest.json describing inputs (portable generator, see tests/_util.py).

Erasure patterns are written out explicitly in the manifest; "bench" = t = r erasures of
information symbols at i * (k // r).
"""
import hashlib
import json
import os
import random
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ORACLE = os.path.join(REPO, "oracle")
SEED = 0x5EED
INLINE_LIMIT = 256 * 1024


def bench_pattern(k, r):
    step = k // r
    return [i * step for i in range(r)]


def rand_pattern(k, r, t, seed, info_only=False):
    rng = random.Random(seed)
    pool = list(range(k if info_only else k + r))
    return sorted(rng.sample(pool, t))


def cases():
    c = []
    def add(name, op, k, r, S, n, t=0, er=(), cosets=None):
        d = dict(name=name, op=op, k=k, r=r, S=S, n=n, seed=SEED, t=t, erased=list(er))
        if cosets is not None:
            d["cosets"] = [list(x) for x in cosets]
        c.append(d)
    # config 1 (k=4, r=2, 256 B) -- full vectors
    add("c1_enc", "encode", 4, 2, 256, 1)
    add("c1_dec_info_rep", "decode", 4, 2, 256, 1, 2, [1, 4])
    add("c1_dec_info2", "decode", 4, 2, 256, 1, 2, [0, 1])
    add("c1_dec_t1", "decode", 4, 2, 256, 1, 1, [2])
    add("c1_dec_toomany", "decode", 4, 2, 256, 1, 3, [0, 1, 2])
    add("kat_iota", "encode_iota", 4, 2, 8, 1)
    # config 2 (k=10, r=4, 4 KiB)
    add("c2_enc", "encode", 10, 4, 4096, 2)
    add("c2_dec_bench", "decode", 10, 4, 4096, 2, 4, bench_pattern(10, 4))
    add("c2_dec_mixed", "decode", 10, 4, 4096, 1, 4, [3, 7, 10, 13])
    add("c2_dec_t3", "decode", 10, 4, 4096, 1, 3, [1, 5, 11])
    # config 3 shape (k=128, r=32) on short symbols; full 64 KiB symbols by hash
    add("c3_enc", "encode", 128, 32, 512, 2)
    add("c3_dec_bench", "decode", 128, 32, 512, 2, 32, bench_pattern(128, 32))
    add("c3_dec_rand17", "decode", 128, 32, 512, 1, 17, rand_pattern(128, 32, 17, 1))
    add("c3_dec_t0", "decode", 128, 32, 512, 1, 0, [])
    add("c3_dec_noncw_bench", "decode_noncw", 128, 32, 512, 1, 32, bench_pattern(128, 32))
    add("c3_dec_noncw_rand", "decode_noncw", 128, 32, 512, 1, 20, rand_pattern(128, 32, 20, 2))
    add("c3_enc_64k", "encode", 128, 32, 65536, 1)
    add("c3_dec_bench_64k", "decode", 128, 32, 65536, 1, 32, bench_pattern(128, 32))
    # config 5 shape (k=4096, r=1024), m = 16
    add("c5_enc", "encode", 4096, 1024, 64, 1)
    add("c5_dec_bench", "decode", 4096, 1024, 64, 1, 1024, bench_pattern(4096, 1024))
    add("c5_dec_rand", "decode", 4096, 1024, 64, 1, 700, rand_pattern(4096, 1024, 700, 3))
    # C5 at full 1 KiB column chunks: the hand-scheduled GF(2^16) kernel (64-byte symbols above only
    # reach the compiled tail kernel); sha256 of the outputs
    add("c5_enc_1k", "encode", 4096, 1024, 1024, 2)
    add("c5_dec_bench_1k", "decode", 4096, 1024, 1024, 1, 1024, bench_pattern(4096, 1024))
    add("c5_dec_rand_2k", "decode", 4096, 1024, 2048, 1, 1024, rand_pattern(4096, 1024, 1024, 9))
    add("c5_dec_t32_1k", "decode", 4096, 1024, 1024, 1, 32, rand_pattern(4096, 1024, 32, 10, info_only=True))
    add("c5_dec_noncw_1k", "decode_noncw", 4096, 1024, 1024, 1, 300, rand_pattern(4096, 1024, 300, 11))
    # round 3: C5 decodes at n = 2 stripes through the bench decode kernels (re-encode decode, plain
    # route), and one-stripe C5 decodes with assorted patterns -- batched together they pin the per-stripe
    # GF(2^16) decode of rsg_decode_batch (every stripe its own pattern; same inputs, stripe 0 of SEED)
    add("c5_dec_bench_1k_n2", "decode", 4096, 1024, 1024, 2, 1024, bench_pattern(4096, 1024))
    add("c5_dec_info1000_1k_n2", "decode", 4096, 1024, 1024, 2, 1000,
        rand_pattern(4096, 1024, 1000, 30, info_only=True))
    add("c5_dec_mixed_1k_n2", "decode", 4096, 1024, 1024, 2, 1024, rand_pattern(4096, 1024, 1024, 31))
    for i, (t, info_only) in enumerate([(1, True), (7, False), (64, False), (333, True), (500, False),
                                        (1000, True), (1023, False), (1024, True)]):
        add(f"c5ps_t{t}_1k", "decode", 4096, 1024, 1024, 1, t, rand_pattern(4096, 1024, t, 40 + i, info_only))
    # the largest codes (k + r = 65535) on whole 1 KiB columns: the GF(2^16) syndrome route and the
    # re-encode decode at maximum n; sha256 of the outputs
    add("max_n_route_enc_1k", "encode", 64511, 1024, 1024, 1)
    add("max_n_route_dec_1k", "decode", 64511, 1024, 1024, 1, 1024,
        rand_pattern(64511, 1024, 1024, 12, info_only=True))
    # example.c shape: 10-byte symbols (5 words, not a multiple of 16 B)
    add("ex_enc", "encode", 100, 10, 10, 1)
    add("ex_dec", "decode", 100, 10, 10, 1, 10, rand_pattern(100, 10, 10, 4))
    # odd symbol sizes: the reference's Release build (-DNDEBUG, the baseline's flags) codes the even
    # prefix, S / 2 words (gf65536.c:158-169), and the written symbols' last byte is zero (fft.c:163
    # memsets each repair symbol, reed_solomon.c:326 each restored one)
    add("odd_enc_9", "encode", 4, 2, 9, 1)
    add("odd_dec_9", "decode", 4, 2, 9, 1, 2, [1, 4])
    add("odd_enc_4097", "encode", 10, 4, 4097, 2)
    add("odd_dec_4097", "decode", 10, 4, 4097, 2, 4, [0, 3, 7, 12])
    # coding matrices via unit vectors (word i of info i = 1)
    add("gmat_4_2", "gmatrix", 4, 2, 8, 1)
    add("gmat_10_4", "gmatrix", 10, 4, 20, 1)
    add("gmat_128_32", "gmatrix", 128, 32, 256, 1)
    add("gmat_4096_1024", "gmatrix", 4096, 1024, 8192, 1)
    add("dmat_128_32_bench", "dmatrix", 128, 32, 320, 1, 32, bench_pattern(128, 32))
    add("dmat_128_32_rand", "dmatrix", 128, 32, 320, 1, 25, rand_pattern(128, 32, 25, 5))
    # edges
    add("edge_r0", "encode", 5, 0, 16, 1)
    add("edge_k0", "encode", 0, 4, 16, 1)
    add("edge_k1r1", "encode", 1, 1, 2, 1)
    add("edge_k1r1_dec", "decode", 1, 1, 2, 1, 1, [0])
    add("edge_repair_only", "decode", 16, 8, 64, 1, 8, list(range(16, 24)))
    add("large_n_enc", "encode", 60000, 16, 4, 1)
    add("large_n_dec", "decode", 60000, 16, 4, 1, 16, rand_pattern(60000, 16, 16, 6))
    add("max_n_enc", "encode", 65519, 16, 2, 1)
    add("wide_r_enc", "encode", 2000, 2000, 4, 1)
    add("wide_r_dec", "decode", 2000, 2000, 4, 1, 2000, rand_pattern(2000, 2000, 2000, 7))
    add("m4_k7r8_enc", "encode", 7, 8, 32, 3)
    add("m8_k200r55_dec", "decode", 200, 55, 32, 2, 40, rand_pattern(200, 55, 40, 8))
    # symbol-wide ops (reference include/rs/gf65536.h:146-167): a = stripe-0 bytes, b = stripe-1 bytes,
    # coefficient in the t field; odd sizes pin the reference's NDEBUG word count (symbol_size / 2)
    add("gf_add_64", "gf_add", 1, 0, 64, 1)
    add("gf_add_odd", "gf_add", 1, 0, 9, 1)
    add("gf_mul_c", "gf_mul", 1, 0, 256, 1, 31981)
    add("gf_mul_0", "gf_mul", 1, 0, 64, 1, 0)
    add("gf_mul_1", "gf_mul", 1, 0, 64, 1, 1)
    add("gf_mul_odd", "gf_mul", 1, 0, 9, 1, 4660)
    add("gf_madd_c", "gf_madd", 1, 0, 256, 1, 12345)
    add("gf_madd_0", "gf_madd", 1, 0, 64, 1, 0)
    add("gf_madd_1", "gf_madd", 1, 0, 64, 1, 1)
    add("gf_madd_odd", "gf_madd", 1, 0, 9, 1, 777)
    # transforms (reference include/rs/fft.h:29-65): f = k symbols, r outputs
    add("fft_t_small", "fft_t", 20, 12, 64, 1)
    add("fft_tc_small", "fft_tc", 20, 12, 64, 1)
    add("fft_tc_r64", "fft_tc", 300, 64, 128, 1)
    add("fft_t_odd", "fft_t", 7, 5, 11, 1)
    add("fft_tc_r1000", "fft_tc", 1100, 1000, 32, 1)
    add("fft_p_small", "fft_p", 16, 10, 64, 1)
    add("fft_p_odd", "fft_p", 9, 6, 11, 1)
    cs = [(0, 1), (21845, 2), (4369, 4), (257, 8), (1, 16), (3, 16)]
    add("fft_pc_mixed", "fft_pc", 40, sum(m for _, m in cs), 64, 1, cosets=cs)
    add("fft_pc_badsize", "fft_pc", 10, 12, 64, 1, cosets=[(1, 8), (5, 4)])  # sizes not the cosets' own
    cs = size16_leaders(64)
    add("fft_pc_c5", "fft_pc", 1024, 1024, 32, 1, cosets=cs)
    return c


def size16_leaders(count):
    """The first `count` leaders (smallest elements) of 2-cyclotomic cosets of size 16 mod 65535."""
    out, x = [], 1
    while len(out) < count:
        rots = {((x << a) | (x >> (16 - a))) & 0xFFFF for a in range(16)}
        if min(rots) == x and len(rots) == 16:
            out.append((x, 16))
        x += 1
    return out


def main():
    subprocess.check_call(["make", "-s", "-C", ORACLE, "ref"])
    gen = os.path.join(ORACLE, "_ref", "gen_golden")
    cs = cases()
    with tempfile.TemporaryDirectory() as tmp:
        spec = os.path.join(tmp, "spec.txt")
        with open(spec, "w") as f:
            for c in cs:
                er = ",".join(map(str, c["erased"])) or "-"
                if "cosets" in c:
                    er = ",".join(f"{l}:{m}" for l, m in c["cosets"])
                f.write(f"{c['name']} {c['op']} {c['k']} {c['r']} {c['S']} {c['n']} {c['seed']} {c['t']} {er}\n")
        out = subprocess.check_output([gen, spec, tmp], text=True)
        rcs = dict(line.split() for line in out.strip().splitlines())
        for c in cs:
            raw = open(os.path.join(tmp, c["name"] + ".bin"), "rb").read()
            c["rc"] = int(rcs[c["name"]])
            c["nbytes"] = len(raw)
            c["sha256"] = hashlib.sha256(raw).hexdigest()
            dst = os.path.join(HERE, c["name"] + ".bin")
            if len(raw) <= INLINE_LIMIT:
                open(dst, "wb").write(raw)
                c["file"] = c["name"] + ".bin"
            elif os.path.exists(dst):
                os.remove(dst)
    meta = dict(generator="oracle/gen_golden.c against oracle/_ref/librs_ref.so "
                          "(reference src/rs + src/memory, -O3 -DNDEBUG)",
                input="tests/_util.py:gen_info (counter-based splitmix64)",
                cases=cs)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"wrote {len(cs)} cases")


if __name__ == "__main__":
    sys.exit(main())
