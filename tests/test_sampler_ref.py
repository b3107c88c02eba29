"""generate()'s sampler chain (koboldcpp_amd/csrc/sampler.h, through the kcpp_sampler_probe test hook) against the
reference's own SampleLogits (gpttype_adapter.cpp:1338-1434), run by oracle/_ref/ref_sampler: the reference file
compiled as one translation unit behind a harness that only feeds it logits, context and parameters
(oracle/ref_sampler.cpp).  Same logits, same mt19937 seed -> the same token, over randomized parameter sets that
cover every sampler, custom orders, rep-pen range / slope / presence, DRY with restart sequences, XTC, dynamic
temperature with smoothing, greedy and both mirostat versions (mirostat starts at the reference's static 2 tau).
No GPU: the probe runs on the host."""
import os
import struct
import subprocess

import numpy as np
import pytest

import koboldcpp_amd.lib as K  # noqa: F401  (loads the library the probe lives in)
from test_sampler import DEFAULT, ORDER_DEFAULT, probe

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "ref_sampler")


@pytest.fixture(scope="module")
def ref():
    if not os.path.exists(REF):
        if not os.path.isdir("/root/reference"):
            pytest.skip("oracle/_ref/ref_sampler not built (reference sources absent)")
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref_sampler"])
    return REF


def pack(logits, P, order, ctx, last_n, restarts, seed, mu=0.0):
    fp = [P["top_k"], P["top_a"], P["top_p"], P["min_p"], P["typical"], P["tfs"], P["temp"], P["rep_pen"],
          P["rep_slope"], P["presence"], P["miro_tau"], P["miro_eta"], P["dry_mult"], P["dry_base"], P["xtc_thr"],
          P["xtc_prob"], P["dyn_range"], P["dyn_exp"], P["smoothing"]]
    ip = [P["rep_range"], P["mirostat"], P["dry_allowed"], P["dry_last_n"]]
    rs = []
    for h, tails in restarts.items():
        for t in tails:
            rs += [h, len(t)] + list(t)
    b = struct.pack("6i", len(logits), P["n_ctx"], len(order), len(ctx), len(last_n), len(rs))
    b += struct.pack("I", seed) + struct.pack("f", mu) + struct.pack("19f", *fp) + struct.pack("4i", *ip)
    for v in (order, ctx, last_n, rs):
        b += struct.pack("%di" % len(v), *v)
    return b + np.ascontiguousarray(logits, dtype=np.float32).tobytes()


def run_ref(ref, blobs):
    out = subprocess.run([ref], input=b"".join(blobs), capture_output=True, check=True, timeout=120).stdout
    return [int(x) for x in out.split()]


def random_case(rng, i):
    P = dict(DEFAULT)
    n = int(rng.choice([300, 2000, 6000]))
    logits = (rng.standard_normal(n) * rng.uniform(0.5, 6.0)).astype(np.float32)
    if i % 5 == 0:                                   # ties and a flat tail
        logits[rng.integers(0, n, n // 3)] = logits.max() - 3.0
    P["temp"] = float(rng.choice([0.0, 0.3, 0.7, 1.0, 1.5])) if i % 7 else 0.0
    if rng.random() < 0.7:
        P["top_k"] = int(rng.choice([0, 1, 5, 40, 100, 300, 1000]))
    if rng.random() < 0.5:
        P["top_p"] = float(rng.uniform(0.5, 1.0))
    if rng.random() < 0.5:
        P["min_p"] = float(rng.uniform(0.0, 0.2))
    if rng.random() < 0.3:
        P["top_a"] = float(rng.uniform(0.0, 0.5))
    if rng.random() < 0.3:
        P["tfs"] = float(rng.uniform(0.8, 1.0))
    if rng.random() < 0.3:
        P["typical"] = float(rng.uniform(0.5, 1.0))
    if rng.random() < 0.5:
        P["rep_pen"] = float(rng.uniform(1.0, 1.5))
        P["rep_slope"] = float(rng.uniform(0.0, 1.5))
        P["presence"] = float(rng.uniform(0.0, 0.5))
        P["rep_range"] = int(rng.choice([0, 16, 64, 320]))
    if rng.random() < 0.4:
        P["dry_mult"] = float(rng.uniform(0.2, 1.5))
        P["dry_base"] = float(rng.uniform(1.1, 2.0))
        P["dry_allowed"] = int(rng.integers(1, 4))
        P["dry_last_n"] = int(rng.choice([0, 50, 200]))
    if rng.random() < 0.3:
        P["xtc_thr"] = float(rng.uniform(0.01, 0.3))
        P["xtc_prob"] = float(rng.uniform(0.3, 1.0))
    if rng.random() < 0.3:
        P["dyn_range"] = float(rng.uniform(0.0, 0.8))
        P["dyn_exp"] = float(rng.uniform(0.5, 2.0))
    if rng.random() < 0.3:
        P["smoothing"] = float(rng.uniform(0.0, 0.6))
    order = list(ORDER_DEFAULT) if rng.random() < 0.6 else [int(x) for x in rng.permutation(7)[: int(rng.integers(3, 8))]]
    vocab_hot = int(rng.integers(20, 80))
    ctx = [int(x) for x in rng.integers(0, vocab_hot, int(rng.integers(50, 500)))]
    ctx += ctx[-30:-6] + ctx[-30:-14]                # repeated spans for DRY / rep-pen
    last_n = ([0] * P["rep_range"] + ctx)[-P["rep_range"]:] if P["rep_range"] > 0 else []
    restarts = {int(rng.integers(0, vocab_hot)): [[]], int(rng.integers(0, vocab_hot)): [[int(rng.integers(0, vocab_hot))]]}
    return logits, P, order, ctx, last_n, restarts


def test_sampler_matches_reference_samplelogits(ref):
    rng = np.random.default_rng(20261017)
    cases, blobs = [], []
    for i in range(160):
        logits, P, order, ctx, last_n, restarts = random_case(rng, i)
        seed = int(rng.integers(0, 2**32 - 1))
        cases.append((logits, P, order, ctx, last_n, restarts, seed))
        blobs.append(pack(logits, P, order, ctx, last_n, restarts, seed))
    want = run_ref(ref, blobs)
    assert len(want) == len(cases)
    got = [probe(lg, P, o, c, ln, rs, sd)[0] for (lg, P, o, c, ln, rs, sd) in cases]
    bad = [i for i in range(len(cases)) if got[i] != want[i]]
    assert not bad, [(i, got[i], want[i], cases[i][1]) for i in bad[:5]]


@pytest.mark.parametrize("mirostat", [1, 2])
@pytest.mark.parametrize("k", range(4))
def test_mirostat_matches_reference_samplelogits(ref, mirostat, k):
    """one process per case: the reference's mirostat mu is a function-static set to 2 tau on its first call"""
    rng = np.random.default_rng(100 * mirostat + k)
    logits, P, order, ctx, last_n, restarts = random_case(rng, 1 + k)
    P.update(mirostat=mirostat, miro_tau=float(rng.uniform(2.0, 8.0)), miro_eta=float(rng.uniform(0.05, 0.3)),
             temp=float(rng.uniform(0.5, 1.2)), dry_mult=0.0)
    seed = int(rng.integers(0, 2**32 - 1))
    want = run_ref(ref, [pack(logits, P, order, ctx, last_n, restarts, seed)])[0]
    got = probe(logits, P, order, ctx, last_n, restarts, seed, mu=2.0 * P["miro_tau"])[0]
    assert got == want


def test_reference_harness_is_sensitive(ref):
    """the comparison is not vacuous: different seeds draw different tokens at temperature, and a rep-pen / DRY
    context moves the reference's greedy pick"""
    rng = np.random.default_rng(5)
    logits = (rng.standard_normal(2000) * 1.0).astype(np.float32)
    P = dict(DEFAULT, temp=1.0)
    toks = run_ref(ref, [pack(logits, P, ORDER_DEFAULT, [1, 2], [], {}, s) for s in range(40)])
    assert len(set(toks)) > 20
    top = int(np.argmax(logits))
    G = dict(DEFAULT, temp=0.0, rep_pen=3.0, rep_range=64)
    assert run_ref(ref, [pack(logits, G, ORDER_DEFAULT, [top] * 10, [top] * 10, {}, 1)]) != [top]
    assert probe(logits, G, ORDER_DEFAULT, [top] * 10, [top] * 10, {}, 1)[0] != top
