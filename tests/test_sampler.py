"""Host-side parity of generate()'s sampler chain (koboldcpp_amd/csrc/sampler.h) with the reference's
SampleLogits (gpttype_adapter.cpp:1338-1434), restated here independently in Python.

Covers the default and custom sampler orders, top-k/top-a/top-p+min-p/tfs/typical/temperature, dynamic
temperature with smoothing, repetition penalty with slope and presence penalty, DRY with restart
sequences, XTC, mirostat v2 and greedy; the final draw restates libstdc++'s std::discrete_distribution over
std::mt19937 (generate_canonical<double, 53>, lower_bound on the normalised partial sums), so the same seed
must give the same token.  No GPU: the probe entry runs on the host."""
import ctypes
import math

import numpy as np
import pytest

import koboldcpp_amd.lib as K

F32 = np.float32


class MT19937:
    """std::mt19937 (init_genrand seeding)"""

    def __init__(self, seed):
        self.mt = [0] * 624
        self.mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            self.mt[i] = (1812433253 * (self.mt[i - 1] ^ (self.mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.i = 624

    def __call__(self):
        if self.i >= 624:
            for k in range(624):
                y = (self.mt[k] & 0x80000000) | (self.mt[(k + 1) % 624] & 0x7FFFFFFF)
                self.mt[k] = self.mt[(k + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            self.i = 0
        y = self.mt[self.i]
        self.i += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF


def canonical_double(rng):
    r = (rng() + rng() * 4294967296.0) / 18446744073709551616.0
    return r if r < 1.0 else math.nextafter(1.0, 0.0)


def canonical_float(rng):
    r = F32(rng() / 4294967296.0)
    return r if r < F32(1.0) else np.nextafter(F32(1.0), F32(0.0))


def discrete(probs, rng):
    """libstdc++ discrete_distribution<int>: probabilities normalised in double, partial sums, last = 1"""
    p = [float(x) for x in probs]
    s = sum(p)
    p = [x / s for x in p]
    cp, acc = [], 0.0
    for x in p:
        acc += x
        cp.append(acc)
    cp[-1] = 1.0
    u = canonical_double(rng)
    lo, hi = 0, len(cp)
    while lo < hi:                      # lower_bound
        mid = (lo + hi) // 2
        if cp[mid] < u:
            lo = mid + 1
        else:
            hi = mid
    return lo


class C:
    """llama_token_data_array: items [id, logit, p] (float32), size, sorted"""

    def __init__(self, logits):
        self.d = [[i, F32(v), F32(0)] for i, v in enumerate(logits)]
        self.sorted = False

    def sort(self):
        if not self.sorted:
            self.d.sort(key=lambda t: -t[1])
            self.sorted = True


def softmax(c):                                    # sample_softmax :483-506
    c.sort()
    mx = c.d[0][1]
    cum = F32(0)
    for t in c.d:
        t[2] = F32(np.exp(F32(t[1] - mx)))
        cum = F32(cum + t[2])
    for t in c.d:
        t[2] = F32(t[2] / cum)


def top_k(c, k):                                   # :508-583 (result = the k largest, sorted)
    if k <= 0:
        k = len(c.d)
    k = min(max(k, 1), len(c.d))
    c.sort()
    c.d = c.d[:k]


def top_a(c, a):                                   # :675-701
    if a <= 0 or len(c.d) <= 1:
        return
    softmax(c)
    thr = F32(F32(a) * c.d[0][2] * c.d[0][2])
    for i, t in enumerate(c.d):
        if t[2] < thr and i >= 1:
            c.d = c.d[:i]
            return


def top_p(c, p):                                   # :1009-1033
    if p >= 1:
        return
    softmax(c)
    cum = F32(0)
    for i, t in enumerate(c.d):
        cum = F32(cum + t[2])
        if cum >= F32(p) and i + 1 >= 1:
            c.d = c.d[:i + 1]
            return


def min_p(c, p):                                   # :1035-1088
    if p <= 0 or not c.d:
        return
    if not c.sorted:
        mx = max(t[1] for t in c.d)
        ml = F32(mx + F32(np.log(F32(p))))
        kept = [t for t in c.d if t[1] >= ml]
        if len(kept) >= 1:
            c.d = kept
            return
    c.sort()
    ml = F32(c.d[0][1] + F32(np.log(F32(p))))
    i = 1
    while i < len(c.d):
        if c.d[i][1] < ml and i >= 1:
            break
        i += 1
    c.d = c.d[:i]


def tail_free(c, z):                               # :1090-1142
    if z >= 1 or len(c.d) <= 2:
        return
    softmax(c)
    d1 = [F32(c.d[i][2] - c.d[i + 1][2]) for i in range(len(c.d) - 1)]
    d2 = [F32(abs(F32(d1[i] - d1[i + 1]))) for i in range(len(d1) - 1)]
    s = F32(0)
    for v in d2:
        s = F32(s + v)
    d2 = [F32(v / s) for v in d2] if s > F32(1e-6) else [F32(1.0 / len(d2))] * len(d2)
    cum = F32(0)
    for i, v in enumerate(d2):
        cum = F32(cum + v)
        if cum > F32(z) and i >= 1:
            c.d = c.d[:i]
            return


def typical(c, p):                                 # :1144-1203
    if p >= 1:
        return
    softmax(c)
    ent = F32(0)
    for t in c.d:
        if t[2] > 0:
            ent = F32(ent + F32(-t[2] * F32(np.log(t[2]))))
    sh = [F32(abs(F32(-F32(np.log(t[2])) - ent))) for t in c.d]
    idx = sorted(range(len(c.d)), key=lambda i: sh[i])
    cum = F32(0)
    last = len(idx)
    for i, j in enumerate(idx):
        cum = F32(cum + c.d[j][2])
        if cum > F32(p) and i >= 0:
            last = i + 1
            break
    c.d = [c.d[j] for j in idx[:last]]
    c.sorted = False


def smooth(c, f):
    softmax(c)
    h = c.d[0][1]
    for t in c.d:
        s = F32(t[1] - h)
        t[1] = F32(F32(-F32(f) * s * s) + h)
    softmax(c)


def temperature(c, temp, smoothing):               # :1265-1296
    greedy = temp <= 0
    if greedy:
        temp, smoothing = 0.00390625, 0
    for t in c.d:
        t[1] = F32(t[1] / F32(temp))
    if smoothing > 0 and len(c.d) > 1:
        smooth(c, smoothing)
    if greedy:
        top_k(c, 1)


def entropy(c, tmin, tmax, expo, smoothing):       # :1205-1263
    if len(c.d) <= 1:
        return
    max_ent = F32(-np.log(F32(1.0) / F32(len(c.d))))
    softmax(c)
    ent = F32(0)
    for t in c.d:
        if t[2] > 0:
            ent = F32(ent - F32(t[2] * F32(np.log(t[2]))))
    dyn = F32(F32(tmin) + F32(F32(tmax) - F32(tmin)) * F32(np.power(F32(ent / max_ent), F32(expo))))
    for t in c.d:
        t[1] = F32(t[1] / dyn)
    mx = float(c.d[0][1])
    ps = [math.exp(float(t[1]) - mx) for t in c.d]
    s = sum(ps)
    for t, v in zip(c.d, ps):
        t[2] = F32(F32(v) / s)
    if smoothing > 0 and len(c.d) > 1:
        smooth(c, smoothing)


def rep_pen(c, n_ctx, rng_, pen, slope, presence, last_n):   # :950-1007
    nrep = min(len(last_n), rng_, n_ctx)
    lt = last_n[len(last_n) - nrep:]
    if nrep == 0 or (pen == 1 and presence == 0):
        return
    near = {lt[i] for i in range(nrep) if 2 * i >= nrep}
    far = {lt[i] for i in range(nrep) if 2 * i < nrep}
    red = F32(1 + (pen - 1) * slope) if pen > 1 else F32(pen)
    for t in c.d:
        if t[0] not in near and t[0] not in far:
            continue
        pv = F32(pen) if t[0] in near else red
        t[1] = F32(t[1] * pv) if t[1] <= 0 else F32(t[1] / pv)
        t[1] = F32(t[1] - F32(presence))
    c.sorted = False


def dry(c, n_ctx, rng_, mult, base, allowed, restarts, ctx):   # :744-948 (naive suffix matching)
    if mult <= 0 or base <= 0:
        return
    if rng_ <= 0 or rng_ > n_ctx:
        rng_ = n_ctx
    nrep = min(len(ctx), rng_, n_ctx)
    if nrep <= allowed:
        return
    lt = ctx[len(ctx) - nrep:]
    rep_limit = nrep
    for i in range(nrep):
        ix = nrep - 1 - i
        tails = restarts.get(lt[ix], [])
        longest = -1
        for tail in tails:
            if longest < len(tail) <= i and all(tail[o] == lt[ix + 1 + o] for o in range(len(tail))):
                longest = len(tail)
        if tails and longest >= 0:
            rep_limit = i - longest
            break
    if rep_limit <= allowed:
        return
    # repeat count at i = length of the common suffix of lt[:i+1] and lt (capped), i < nrep-1
    maxrep = {}
    for i in range(nrep - 1):
        n = 0
        while n <= i and lt[i - n] == lt[nrep - 1 - n]:
            n += 1
        n = min(n, rep_limit)
        if n >= allowed:
            tok = lt[i + 1]
            if maxrep.get(tok, -1) < n:
                maxrep[tok] = n
    max_exp = int(88.7228391 / math.log(base)) if base > 1.000001 else 0
    for tok, n in maxrep.items():
        e = n - allowed
        if max_exp > 0 and e > max_exp:
            e = max_exp
        t = c.d[tok]
        t[1] = F32(t[1] - F32(mult * float(F32(base)) ** e))
    if maxrep:
        c.sorted = False


def xtc(c, thr, prob, rng):                        # :703-742
    if thr > 0.5 or prob <= 0 or len(c.d) <= 1:
        return
    if canonical_float(rng) >= F32(prob):
        return
    softmax(c)
    last = len(c.d)
    for i, t in enumerate(c.d):
        if t[2] < F32(thr):
            last = i
            break
    if last > 1:
        for t in c.d[:last - 1]:
            t[1] = F32(t[1] - F32(999))
        c.sorted = False


def chain(logits, P, order, ctx, last_n, restarts, seed):
    """SampleLogits (non-mirostat): returns (candidates after the chain with their draw probabilities, token)"""
    rng = MT19937(seed)
    c = C(logits)
    dry(c, P["n_ctx"], P["dry_last_n"], P["dry_mult"], P["dry_base"], P["dry_allowed"], restarts, ctx)
    top_k(c, 5000)
    for s in order:
        if s == 0:
            top_k(c, int(P["top_k"]))
        elif s == 1:
            top_a(c, P["top_a"])
        elif s == 2:
            top_p(c, P["top_p"])
            min_p(c, P["min_p"])
        elif s == 3:
            tail_free(c, P["tfs"])
        elif s == 4:
            typical(c, P["typical"])
        elif s == 5:
            if P["dyn_range"] > 0:
                entropy(c, max(0.0, P["temp"] - P["dyn_range"]), max(0.0, P["temp"] + P["dyn_range"]),
                        max(0.0, P["dyn_exp"]), P["smoothing"])
            else:
                temperature(c, P["temp"], P["smoothing"])
        elif s == 6:
            rep_pen(c, P["n_ctx"], P["rep_range"], P["rep_pen"], P["rep_slope"], P["presence"], last_n)
    xtc(c, P["xtc_thr"], P["xtc_prob"], rng)
    softmax(c)
    k = discrete([t[2] for t in c.d], rng)
    return c.d, c.d[k][0]


DEFAULT = dict(top_k=0, top_a=0, top_p=1, min_p=0, typical=1, tfs=1, temp=1, rep_pen=1, rep_slope=1, presence=0,
               miro_tau=5, miro_eta=0.1, dry_mult=0, dry_base=0, xtc_thr=0, xtc_prob=0, dyn_range=0, dyn_exp=1,
               smoothing=0, rep_range=64, mirostat=0, dry_allowed=2, dry_last_n=0, n_ctx=2048)
ORDER_DEFAULT = [6, 0, 1, 3, 4, 2, 5]


def probe(logits, P, order, ctx, last_n, restarts, seed, mu=0.0):
    L = K.raw()
    fp = (ctypes.c_float * 19)(P["top_k"], P["top_a"], P["top_p"], P["min_p"], P["typical"], P["tfs"], P["temp"],
                               P["rep_pen"], P["rep_slope"], P["presence"], P["miro_tau"], P["miro_eta"], P["dry_mult"],
                               P["dry_base"], P["xtc_thr"], P["xtc_prob"], P["dyn_range"], P["dyn_exp"], P["smoothing"])
    ip = (ctypes.c_int * 4)(P["rep_range"], P["mirostat"], P["dry_allowed"], P["dry_last_n"])
    rs = []
    for h, tails in restarts.items():
        for t in tails:
            rs += [h, len(t)] + list(t)
    arr = lambda v, t=ctypes.c_int: (t * max(1, len(v)))(*v)
    lg = np.ascontiguousarray(logits, dtype=np.float32)
    cap = len(logits)
    ids = (ctypes.c_int * cap)()
    ps = (ctypes.c_float * cap)()
    n = ctypes.c_int(0)
    m = ctypes.c_float(mu)
    tok = L.kcpp_sampler_probe(lg.ctypes.data_as(ctypes.c_void_p), len(lg), P["n_ctx"], fp, ip, arr(order), len(order),
                               arr(ctx), len(ctx), arr(last_n), len(last_n), arr(rs), len(rs), seed, ctypes.byref(m),
                               ids, ps, cap, ctypes.byref(n))
    return tok, [(ids[i], ps[i]) for i in range(n.value)], m.value


def _logits(seed, n=600, scale=3.0):
    return (np.random.default_rng(seed).standard_normal(n) * scale).astype(np.float32)


CASES = [
    ("default_order", dict(temp=0.8, top_k=40, top_p=0.9, min_p=0.05, rep_pen=1.1, rep_slope=0.7, presence=0.2),
     ORDER_DEFAULT),
    ("temp_first", dict(temp=1.3, typical=0.9, tfs=0.95, top_a=0.2), [5, 4, 3, 1, 0, 2, 6]),
    ("dynatemp_smoothing", dict(temp=1.0, dyn_range=0.5, dyn_exp=1.3, smoothing=0.3, top_k=200), ORDER_DEFAULT),
    ("dry", dict(temp=0.9, dry_mult=0.8, dry_base=1.75, dry_allowed=2, dry_last_n=0), ORDER_DEFAULT),
    ("xtc", dict(temp=1.0, xtc_thr=0.05, xtc_prob=1.0, top_k=50), ORDER_DEFAULT),
    ("greedy", dict(temp=0.0, rep_pen=1.2), ORDER_DEFAULT),
    ("topk_bucket", dict(temp=0.7, top_k=300, top_p=0.97), [0, 5, 2]),
]


@pytest.mark.parametrize("name,over,order", CASES, ids=[c[0] for c in CASES])
def test_sampler_chain_matches_reference_restatement(name, over, order):
    P = dict(DEFAULT)
    P.update(over)
    logits = _logits(hash(name) % 1000)
    ctx = [int(x) for x in np.random.default_rng(7).integers(0, 40, 300)]
    ctx += ctx[-25:-5] + ctx[-25:-12]                           # a repeated span for DRY / rep_pen
    last_n = ([0] * P["rep_range"] + ctx)[-P["rep_range"]:]
    restarts = {3: [[]], 11: [[12, 13]]}
    for seed in (1, 42, 123456):
        ref_c, ref_tok = chain(logits, P, order, ctx, last_n, restarts, seed)
        tok, cands, _ = probe(logits, P, order, ctx, last_n, restarts, seed)
        assert [i for i, _ in cands] == [t[0] for t in ref_c], name
        np.testing.assert_allclose([p for _, p in cands], [float(t[2]) for t in ref_c], rtol=2e-5, atol=1e-7)
        assert tok == ref_tok, (name, seed)


def test_mirostat_v2_matches_reference_restatement():
    P = dict(DEFAULT, mirostat=2, temp=1.0, miro_tau=4.0, miro_eta=0.2)
    logits = _logits(99)
    for seed in (5, 6, 7):
        mu0 = 2.0 * P["miro_tau"]
        # restated sample_token_mirostat_v2 (:645-671) after rep_pen + temperature
        rng = MT19937(seed)
        c = C(logits)
        top_k(c, 5000)
        temperature(c, P["temp"], 0)
        softmax(c)
        n = 0
        while n < len(c.d) and not (-np.log2(c.d[n][2]) > mu0):
            n += 1
        c.d = c.d[:max(n, 1)]
        softmax(c)
        softmax(c)
        k = discrete([t[2] for t in c.d], rng)
        X = c.d[k][0]
        mu_ref = F32(F32(mu0) - F32(P["miro_eta"]) * F32(F32(-np.log2(c.d[k][2])) - F32(P["miro_tau"])))
        tok, _, mu = probe(logits, P, [], [], [0] * 64, {}, seed, mu=mu0)
        assert tok == X
        assert abs(mu - float(mu_ref)) < 1e-5
