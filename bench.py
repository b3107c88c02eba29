"""Benchmark: Llama-3-8B Q4_K_M (synthetic weights), 4k context, koboldcpp --benchmark semantics.

Workload (BASELINE.json configs[1]): prompt of 3840 tokens prefilled in
ubatches of 512, then greedy decode at positions 3840..4095.  A "step" is one decode token
(one pass of the token-generation hot path); `value` = decode tokens/s.  Prefill tok/s is reported
beside it.  Multi-GPU (--gpus N > 1, with or without torchrun): rank 0 runs load_model's in-process
engine over the N GPUs (layer split by tensor_split 1:...:1, stage streams handing the residual over
by RCCL send/recv, the greedy token moved home to stage 0 by a device copy); the other ranks only
bracket the run with barriers.  value = tokens/s of the whole pipeline.

Adds:
  roofline     -- dominant decode kernel (Q4_K gate|up mat-vec, 4096 x 2*14336), HIP-event timed
  cpu_baseline -- the REFERENCE ggml CPU path (oracle/_ref/ref_llama, built from the reference
                  sources) on the same synthetic 8B weights, bounded sample, rank 0 only.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

LLAMA3_8B = dict(n_vocab=128256, n_embd=4096, n_head=32, n_head_kv=8, n_layer=32, n_ff=14336, n_ctx=4096,
                 eps=1e-5, rope_base=500000.0)
MIXTRAL_8X7B = dict(n_vocab=32000, n_embd=4096, n_head=32, n_head_kv=8, n_layer=32, n_ff=14336, n_ctx=4096,
                    eps=1e-5, rope_base=1000000.0, n_expert=8, n_expert_used=2)
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md chip table (spec)
MFMA_F16_PEAK_TFLOPS = 2500.0   # dense f16 MFMA peak (spec, no sparsity)
MFMA_I8_PEAK_TOPS = 5000.0      # dense i8 MFMA peak: 2x the f16 rate per clock (MI355X_MICROARCH.md, Matrix cores: I8 row)


def q4_k_m_types(n_layer):
    import refharness as R
    return R.q4_k_m_types(n_layer)


def weight_bytes(hp, types):
    import refharness as R
    return sum(R.row_bytes(t, k) * n for (k, n), t in zip(R.weight_shapes(hp), types))


def pmc_traffic():
    """HBM bytes per launch of the roofline kernel from the newest committed PMC summary
    (profiles/rNN_roofline_pmc.json, written by tools/profile_round.sh + tools/roofline_summary.py:
    separate FETCH_SIZE and WRITE_SIZE passes over `bench.py --roofline-only`, FETCH_SIZE doubled per
    the gfx950 correction).  None when no summary exists."""
    import glob
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_roofline_pmc.json")))
    if not fs:
        return None, None
    with open(fs[-1]) as f:
        d = json.load(f)
    return d.get("traffic_bytes_per_launch"), os.path.relpath(fs[-1], ROOT)


def measure_roofline(K, torch, iters=64, pairs=8):
    """Time the dominant decode kernel as the decode path launches it: the fused Q4_K gate|up
    mat-vec over the row-major decode layout with rms_norm+Q8_K prologue and SiLU-GLU epilogue
    (kcpp_gemv_dec(Q4_K_RS, mode 1, pro 1) -> k_gemv_rs, 4096 -> 2 x 14336), HIP events on the launch stream.  Algorithmic bytes per launch =
    both weight matrices + x + norm weight + output row ("roofline")."""
    Kd, N = 4096, 14336
    wbytes = Kd // 256 * 144 * N
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    # 8 weight pairs (8 x 66 MB = 504 MiB, twice the 256 MiB Infinity Cache) so no launch finds its weights cached
    ws = []
    for i in range(pairs):
        a = torch.empty(wbytes, dtype=torch.uint8, device="cuda")
        b = torch.empty(wbytes, dtype=torch.uint8, device="cuda")
        K.call("kcpp_weight_synth", K.Q4_K_RS, 1, 10 + 2 * i, a.data_ptr(), Kd, N, sp)
        K.call("kcpp_weight_synth", K.Q4_K_RS, 1, 11 + 2 * i, b.data_ptr(), Kd, N, sp)
        ws.append((a, b))
    x = torch.randn(Kd, device="cuda")
    nw = torch.ones(Kd, device="cuda")
    y = torch.empty(N, device="cuda")
    args = []
    for a, b in ws:
        d = K.DecArgs()
        d.K, d.x, d.nw, d.eps, d.nseg = Kd, x.data_ptr(), nw.data_ptr(), 1e-5, 1
        d.W[0], d.W2, d.N[0], d.Y[0] = a.data_ptr(), b.data_ptr(), N, y.data_ptr()
        args.append(d)
    for i in range(2 * pairs):
        assert K.gemv_dec(K.Q4_K_RS, args[i % pairs], 1, 1, 1, sp) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for i in range(iters):
        K.gemv_dec(K.Q4_K_RS, args[i % pairs], 1, 1, 1, sp)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    alg = 2 * wbytes + 2 * Kd * 4 + N * 4
    gbs = alg / (ms * 1e-3) / 1e9
    traffic, tsrc = pmc_traffic()
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
            "kernel": "kcpp_gemv_dec -> k_gemv_rs<Q4_K_RS,NI2,R1,GLU,norm+quant prologue,PF,8 waves> 4096x(2x14336)", "bytes_per_launch": alg,
            "avg_us": round(ms * 1e3, 2)}


def cpu_baseline(hp, types, threads, depth=3840, n_ub=512, n_gen=32, threads2=8):
    """The REFERENCE ggml CPU build on the same synthetic weights, koboldcpp --benchmark semantics, on bounded samples:
    (1) at the GPU line's context depth: the prompt's last ubatch (positions depth-512..depth-1, attending over the
    whole prefix) and then n_gen greedy tokens at context depth..depth+n_gen; the earlier prompt positions are taken
    as already cached (zeroed K/V, not computed: REF_SKIP_PREFIX in oracle/ref_llama.c) since a step's cost depends
    on the cache length, not its contents; `threads` = the box's CPU share (16, OMP_NUM_THREADS);
    (2) a 512-token prompt from position 0 and n_gen tokens at context 512..527 at 8 threads."""
    import refharness as R
    if not R.ref_available():
        return None
    prompt = [16 + (i % 2) for i in range(depth)]     # " 1" style repeated ids
    hp2 = dict(hp)
    hp2["n_ctx"] = depth + n_gen + 8
    _, info = R.run_ref_llama(hp2, types, 1234, prompt, n_gen, nthreads=threads, ubatch=n_ub, timeout=900,
                              skip_prefix=depth - n_ub)
    hp3 = dict(hp)
    hp3["n_ctx"] = n_ub + n_gen + 8
    _, info2 = R.run_ref_llama(hp3, types, 1234, prompt[:n_ub], n_gen, nthreads=threads2, ubatch=n_ub, timeout=900)
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except Exception:
        pass
    return {"value": round(n_gen / info["decode_s"], 3), "unit": "tok/s (decode)", "cores": threads,
            "cpu_model": cpu, "host_cpus": os.cpu_count(),
            "cores_reason": "the GPU box grants this job a 16-CPU share (OMP_NUM_THREADS=16 there; nproc shows the whole "
                            "host's CPUs, which other jobs use): more threads would time contention with them, not the "
                            "reference; the 8-thread line is SURVEY.md 8d's setting",
            "kind": "reference",
            "context_depth": [depth, depth + n_gen],
            "prefill_tok_s_last_ubatch": round(n_ub / info["prefill_s"], 3),
            "at_%d_threads_ctx_%d" % (threads2, n_ub): {"decode_tok_s": round(n_gen / info2["decode_s"], 3),
                                                       "prefill_tok_s": round(n_ub / info2["prefill_s"], 3)},
            "sample": "reference ggml CPU (oracle/_ref/ref_llama, built from the reference sources) on the same synthetic "
                      "Llama-3-8B Q4_K_M: the prompt's last %d-token ubatch at positions %d-%d (prefix cached, not "
                      "computed) then %d greedy decode tokens at context %d-%d, %d threads; and a %d-token prompt + %d "
                      "tokens from position 0 at %d threads" % (n_ub, depth - n_ub, depth - 1, n_gen, depth, depth + n_gen,
                                                                threads, n_ub, n_gen, threads2)}


def generate_path(hp, types, n_prompt, n_gen, ubatch, seed=1234):
    """The drop-in number: koboldcpp --benchmark (koboldcpp.py:4274-4348) through the C ABI koboldcpp.py binds --
    load_model() on a full-size Llama-3-8B Q4_K_M GGUF, then ONE generate() with the benchmark's sampler settings
    (temperature 0.1, top_k 1, rep_pen 1, EOS banned), the prompt cut to max_context_length - max_length tokens, and
    koboldcpp's own speeds from get_last_process_time / get_last_eval_time (ms per token, gpttype_adapter.cpp:
    3513-3526).  generate() reads every token's logits on the host and samples there, as the reference does.  The GGUF
    holds the real tensor directory with its data left as a sparse-file hole (no checkpoints exist offline); the
    weights are the runtime's synthetic ones (kcpp_expose_synth_weights), as in the rest of this bench."""
    import ctypes
    import tempfile
    import gguf_writer as GW
    import koboldcpp_amd.lib as K
    from koboldcpp_amd import expose as X
    max_ctx = n_prompt + n_gen
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "llama3-8b-q4_k_m-synthetic.gguf")
        GW.llama_gguf(path, dict(hp, n_ctx=8192), types, seed, GW.WORDS, sparse=True)
        h = X.init_library()
        li = X.load_model_inputs()
        li.model_filename = path.encode()
        li.max_context_length = max_ctx
        li.blasbatchsize = ubatch
        li.gpulayers = 999
        li.flash_attention = True
        li.rope_freq_base = 10000.0
        li.rope_freq_scale = 0.0          # koboldcpp.py default --ropeconfig: the model's own RoPE
        if not h.load_model(li):
            raise RuntimeError("load_model failed")
        if K.raw().kcpp_expose_synth_weights(ctypes.c_uint64(seed)) != 0:
            raise RuntimeError("kcpp_expose_synth_weights failed")

        def gen(prompt, n):
            # the request koboldcpp.py's generate() builds for its --benchmark call (koboldcpp.py:870-1000): the
            # benchmark's temperature 0.1 / top_k 1 / rep_pen 1 / ban_eos_token, every other field at its default
            gi = X.generation_inputs()
            gi.prompt, gi.memory = prompt, b""
            gi.max_context_length, gi.max_length = max_ctx, n
            gi.temperature, gi.top_k, gi.rep_pen, gi.seed = 0.1, 1, 1.0, 7
            gi.top_a, gi.top_p, gi.min_p, gi.typical_p, gi.tfs = 0.0, 0.92, 0.0, 1.0, 1.0
            gi.rep_pen_range, gi.rep_pen_slope, gi.presence_penalty = 320, 1.0, 0.0
            gi.mirostat, gi.mirostat_tau, gi.mirostat_eta = 0, 5.0, 0.1
            gi.dry_multiplier, gi.dry_base, gi.dry_allowed_length, gi.dry_penalty_last_n = 0.0, 1.75, 2, 320
            gi.xtc_threshold, gi.xtc_probability = 0.2, 0.0
            gi.dynatemp_range, gi.dynatemp_exponent, gi.smoothing_factor = 0.0, 1.0, 0.0
            for i, v in enumerate([6, 0, 1, 3, 4, 2, 5]):
                gi.sampler_order[i] = v
            gi.sampler_len = 7
            gi.allow_eos_token, gi.bypass_eos_token = False, False      # ban_eos_token = True
            out = h.generate(gi)
            if out.status != 1:
                raise RuntimeError("generate failed")
            return h.get_last_token_count()
        gen(b"hello world", 8)                      # warm-up (first touch, graph capture); shares only BOS
        # the benchmark prompt (" 1" repeated, koboldcpp.py:4300-4303), long enough to be cut to n_prompt tokens
        n = gen(b" 1" * (n_prompt + 64), n_gen)
        pt, et = h.get_last_process_time(), h.get_last_eval_time()
    return {"decode_tok_s": round(1000.0 / et, 2), "prefill_tok_s": round(1000.0 / pt, 1), "gen_tokens": n,
            "max_context_length": max_ctx,
            "how": "koboldcpp --benchmark semantics through the C ABI: load_model (sparse full-size GGUF, synthetic "
                   "weights) + one generate() with the request koboldcpp.py builds (temperature 0.1, top_k 1, rep_pen 1, "
                   "EOS banned, other samplers at their defaults: the chain reduces to the argmax, so each step's own "
                   "device argmax is read back; the token returns to the host every step); speeds = 1000 / "
                   "get_last_eval_time and 1000 / get_last_process_time (ms per token)"}


def run_model(K, torch, hp, types, n_prompt, ubatch, steps, warmup):
    """koboldcpp --benchmark semantics on one GPU: prefill n_prompt ids (" 1" pattern) in ubatches, then
    greedy decode (graph replay + on-device argmax per token).  Weights and inputs resident before timing."""
    m = K.Model(hp, types, max_ubatch=ubatch)
    m.synth(1234)
    prompt = [16 + (i % 2) for i in range(n_prompt)]
    # warm-up prefill on a short prompt (first touch of buffers / graph capture)
    m.decode(prompt[:64], 0, want_logits=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.decode(prompt, 0, want_logits=False)
    torch.cuda.synchronize()
    t_pp = time.perf_counter() - t0
    m.argmax()                            # first generated token; stays on device for the next step
    n_past = len(prompt)
    for _ in range(warmup):
        m.decode_greedy(n_past)
        n_past += 1
    steps = min(steps, hp["n_ctx"] - n_past)
    torch.cuda.synchronize()
    # every token comes back to the host, one step behind the device (the next step is queued while the host reads
    # the previous token: kcpp_model_decode_greedy_lagged); the timed region ends when the last token is on the host
    toks = []
    t0 = time.perf_counter()
    for _ in range(steps):
        toks.append(m.decode_greedy_lagged(n_past))
        n_past += 1
    toks.append(m.greedy_drain())
    torch.cuda.synchronize()
    t_tg = time.perf_counter() - t0
    assert toks[0] == -1 and min(toks[1:]) >= 0 and len(toks) == steps + 1
    wb = m.weight_bytes()
    m.close()
    return {"dec": steps / t_tg, "pre": n_prompt / t_pp, "t_pp": t_pp, "ms_step": t_tg / steps * 1e3, "steps": steps,
            "n_past": n_past, "wb": wb}


def other_config(args, K, torch):
    """BASELINE configs[2] (Llama-3-8B all-Q8_0, prefill in ubatches of 32: the batched MFMA mat-mul path,
    HBM-bound at 32 tokens) and configs[4] (Mixtral-8x7B-shape Q5_K_M, 8 experts top-2:
    expert-routed decode mat-vecs).  Parity-tested at small sizes in tests/; these are their measurements."""
    import refharness as R
    if args.config == "llama3-8b-q8_0-b32":
        hp = dict(LLAMA3_8B)
        types = R.uniform_types(hp["n_layer"], R.Q8_0)
        n_prompt, ub = (args.prompt if args.prompt != 3840 else 1024), 32
        r = run_model(K, torch, hp, types, n_prompt, ub, min(args.steps, 64), args.warmup)
        # bytes per ubatch: every layer weight once (the Q8_0 output head runs once per llama_decode call)
        shapes = R.weight_shapes(hp)
        layer_bytes = sum(R.row_bytes(t, k) * n for i, ((k, n), t) in enumerate(zip(shapes, types)) if i >= 3)
        n_ub = -(-n_prompt // ub)
        t_ub = r["t_pp"] / n_ub
        gbs = layer_bytes / t_ub / 1e9
        flops = 2 * sum(k * n for i, (k, n) in enumerate(shapes) if i >= 3 and n > 1) * ub
        return {"metric": "prefill tok/s at ubatch 32 (Llama-3-8B Q8_0)", "value": round(r["pre"], 1), "unit": "tok/s",
                "n_gpus": 1, "higher_is_better": True,
                "dtype": "q8_0 weights x q8_0 activations (exact int8 block dots on i8 MFMA, f32 combination)", "data": "synthetic",
                "config": {"workload": "llama3-8b-q8_0 prefill %d tokens in ubatches of %d" % (n_prompt, ub),
                           "model": "Llama-3-8B-shape Q8_0 random-init", "parallelism": "single GPU"},
                "ms_per_ubatch": round(t_ub * 1e3, 3), "decode_tok_s": round(r["dec"], 2),
                "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_ubatch": layer_bytes,
                             "mfma_TFLOPs": round(flops / t_ub / 1e12, 1), "scope": "whole ubatch (all layers)"}}
    if args.config == "mixtral-8x7b-q5_k_m":
        hp = dict(MIXTRAL_8X7B)
        types = R.mixtral_q5_k_m_types(hp["n_layer"])
        n_prompt = args.prompt if args.prompt != 3840 else 512
        r = run_model(K, torch, hp, types, n_prompt, args.ubatch, args.steps, args.warmup)
        shapes = R.weight_shapes(hp)
        tok_bytes = 0
        for i, ((k, n), t) in enumerate(zip(shapes, types)):
            if i == 0:
                continue                   # token embedding: one row gathered
            b = R.row_bytes(t, k) * n
            tok_bytes += b * (hp["n_expert_used"] if R.n_slices(hp, i) > 1 else 1)
        kv = 2 * hp["n_layer"] * hp["n_head_kv"] * (hp["n_embd"] // hp["n_head"]) * 2 * (r["n_past"] - r["steps"] / 2)
        gbs = (tok_bytes + kv) / (r["ms_step"] * 1e-3) / 1e9
        return {"metric": "decode tok/s (Mixtral-8x7B Q5_K_M, top-2 of 8 experts)", "value": round(r["dec"], 2),
                "unit": "tok/s", "n_gpus": 1, "steps": r["steps"], "warmup": args.warmup,
                "ms_per_step": round(r["ms_step"], 4), "higher_is_better": True,
                "dtype": "q5_K/q6_K/q8_0 weights x q8_K/q8_0 activations; f16 KV", "data": "synthetic",
                "config": {"workload": "mixtral-8x7b-q5_k_m: prefill %d + greedy decode" % n_prompt,
                           "model": "Mixtral-8x7B-shape Q5_K_M random-init", "parallelism": "single GPU"},
                "prefill_tok_s": round(r["pre"], 1), "weight_bytes": r["wb"], "bytes_per_token": tok_bytes,
                "decode_effective_GBps": round(gbs, 1), "decode_hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}
    if args.config == "llama3-70b-stage":
        return stage70b(args, K, torch)
    raise SystemExit("unknown --config %s" % args.config)


LLAMA3_70B = dict(n_vocab=128256, n_embd=8192, n_head=64, n_head_kv=8, n_layer=80, n_ff=28672, n_ctx=4096,
                  eps=1e-5, rope_base=500000.0)


def stage70b(args, K, torch):
    """BASELINE configs[3] (Llama-3-70B Q4_K_M, --tensorsplit over 8 GPUs) as one GPU can measure it: the first
    pipeline stage exactly as load_model builds it for tensor_split 1:...:1 (layers [0, 10) + the embedding), 4k
    context (prefill 3840 in ubatches of 512, then single-token steps at 3841..), its decode rate and HBM fraction;
    and the per-boundary cost of the stage hand-off, from the 8B bench model run as 1 stage and as 8 stages on this
    one GPU (KCPP_VIRTUAL_DEVICES: the event-ordered device-copy hand-off of expose.cpp, 7 hidden-state hops + the
    token home per step).  The 8-GPU curve itself is the driver's (SCALE)."""
    import refharness as R
    hp = dict(LLAMA3_70B)
    types = R.q4_k_m_types(hp["n_layer"])
    il1 = hp["n_layer"] // 8
    m = K.Model(hp, types, il0=0, il1=il1, has_embed=True, has_output=False, max_ubatch=args.ubatch)
    m.synth(1234)
    prompt = [16 + (i % 2) for i in range(args.prompt)]
    m.decode(prompt[:64], 0, want_logits=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.decode(prompt, 0, want_logits=False)
    torch.cuda.synchronize()
    t_pp = time.perf_counter() - t0
    n = len(prompt)
    m.decode([16], n, want_logits=False)        # the stage's single-token graph; its token stays in tok_dev
    n += 1
    L = K.raw()
    for _ in range(args.warmup):
        assert L.kcpp_model_step_dev(m.m, n) == 0
        n += 1
    steps = min(args.steps, hp["n_ctx"] - n)
    m.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        assert L.kcpp_model_step_dev(m.m, n) == 0
        n += 1
    m.sync()
    t_tg = time.perf_counter() - t0
    wb = m.weight_bytes()
    m.close()
    embd = R.row_bytes(types[0], hp["n_embd"]) * hp["n_vocab"]
    kv = 2 * il1 * hp["n_head_kv"] * (hp["n_embd"] // hp["n_head"]) * 2 * (n - steps / 2)
    tok_bytes = wb - embd + kv
    ms = t_tg / steps * 1e3
    gbs = tok_bytes / (ms * 1e-3) / 1e9
    # hand-off cost: the 8B bench model as 1 stage vs 8 stages on this GPU (same work, 8 hops more per step)
    hp8, t8 = dict(LLAMA3_8B), q4_k_m_types(32)
    hs = min(64, args.steps)
    os.environ["KCPP_VIRTUAL_DEVICES"] = "1"
    try:
        one = K.engine_bench(hp8, t8, 1, 512, 512, 8, hs)
        eight = K.engine_bench(hp8, t8, 8, 512, 512, 8, hs)
    finally:
        del os.environ["KCPP_VIRTUAL_DEVICES"]
    per_hop_us = (eight["decode_s"] - one["decode_s"]) / hs / 8 * 1e6
    return {"metric": "decode tok/s of one Llama-3-70B Q4_K_M pipeline stage (layers 0-9 + embedding, 4k ctx)",
            "value": round(1e3 / ms, 2), "unit": "tok/s", "n_gpus": 1, "steps": steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 4), "higher_is_better": True,
            "dtype": "q4_K/q6_K weights x q8_K activations (int8 dot, f32 accum); f16 KV", "data": "synthetic",
            "config": {"workload": "llama3-70b-q4_k_m stage [0,%d) of tensor_split 1:...:1 over 8 GPUs: prefill %d "
                                   "(ubatch %d) + single-token steps" % (il1, args.prompt, args.ubatch),
                       "model": "Llama-3-70B-shape Q4_K_M random-init", "parallelism": "one pipeline stage on one GPU"},
            "prefill_tok_s": round(args.prompt / t_pp, 1), "stage_bytes_per_token": int(tok_bytes),
            "decode_effective_GBps": round(gbs, 1), "decode_hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
            "handoff": {"per_hop_us": round(per_hop_us, 2), "hops_per_step": 8,
                        "one_stage_ms_per_token": round(one["decode_s"] / hs * 1e3, 4),
                        "eight_stages_ms_per_token": round(eight["decode_s"] / hs * 1e3, 4),
                        "how": "Llama-3-8B bench model, 512-token prompt, %d greedy steps: 1 stage vs 8 stages on one GPU "
                               "(KCPP_VIRTUAL_DEVICES, event-ordered device copies); (t8 - t1) / steps / 8 hops "
                               "(7 hidden states + the token home)" % hs}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=3840)
    ap.add_argument("--ubatch", type=int, default=512)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-generate-path", action="store_true",
                    help="skip the generate() leg (koboldcpp --benchmark through the C ABI)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the dominant-kernel timing (for the rocprofv3 --pmc passes in profiles/)")
    ap.add_argument("--config", default="llama3-8b-q4_k_m",
                    choices=["llama3-8b-q4_k_m", "llama3-8b-q8_0-b32", "mixtral-8x7b-q5_k_m", "llama3-70b-stage"],
                    help="BASELINE configs[1] (default: the driver's line), configs[2], configs[4], configs[3]'s one-GPU stage")
    ap.add_argument("--layers", type=int, default=None, help="override n_layer (debug only; invalidates metric)")
    args = ap.parse_args()

    import torch
    import koboldcpp_amd.lib as K

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    n_dev = max(args.gpus, world)
    if n_dev > 1 and torch.cuda.device_count() < n_dev:     # device_count does not initialise the GPU here
        raise SystemExit("bench.py: --gpus %d but %d GPU(s) visible" % (n_dev, torch.cuda.device_count()))
    if world > 1:
        # launched by torchrun: the multi-GPU path is the in-process engine on rank 0 over all world GPUs (what
        # load_model ships); the other ranks touch no GPU and only bracket the run with (gloo) barriers, so the
        # max-over-ranks time is rank 0's
        import torch.distributed as dist
        dist.init_process_group("gloo")
        dist.barrier()
        if rank == 0:
            run_bench(args, K, torch, n_dev)
        dist.barrier()
        dist.destroy_process_group()
        return
    run_bench(args, K, torch, n_dev)


def run_bench(args, K, torch, n_dev):
    torch.cuda.set_device(0)
    if args.roofline_only:
        print(json.dumps({"roofline": measure_roofline(K, torch)}))
        return
    if args.config != "llama3-8b-q4_k_m":
        print(json.dumps(other_config(args, K, torch)))
        return
    hp = dict(LLAMA3_8B)
    if args.layers:
        hp["n_layer"] = args.layers
    types = q4_k_m_types(hp["n_layer"])
    if n_dev == 1:
        r = run_model(K, torch, hp, types, args.prompt, args.ubatch, args.steps, args.warmup)
        par = "single GPU"
    else:
        # the drop-in engine load_model ships (koboldcpp_amd/csrc/expose.cpp): n_dev layer-split stages in this one
        # process, RCCL send/recv hand-off between the stage streams, pipelined prefill ubatches, greedy steps with
        # the argmax on the last stage and the token moved home to stage 0 by a 4-byte device copy (expose.cpp
        # greedy_step / token_home: no host synchronisation inside a step)
        steps = min(args.steps, hp["n_ctx"] - args.prompt - args.warmup - 1)
        e = K.engine_bench(hp, types, n_dev, args.prompt, args.ubatch, args.warmup, steps)
        r = {"dec": steps / e["decode_s"], "pre": args.prompt / e["prefill_s"], "t_pp": e["prefill_s"],
             "ms_step": e["decode_s"] / steps * 1e3, "steps": steps, "n_past": e["n_past"], "wb": weight_bytes(hp, types)}
        par = "layer split over %d GPUs (tensor_split 1:...:1), %s hand-off, one process" % (
            n_dev, "RCCL send/recv" if e["rccl"] else "event-ordered peer copy")
    print(json.dumps(bench_line(args, K, torch, hp, types, r, n_dev, par)))


def bench_line(args, K, torch, hp, types, r, n_dev, par):
    dec, pre, ms_step, steps, n_past, wb, t_pp = r["dec"], r["pre"], r["ms_step"], r["steps"], r["n_past"], r["wb"], r["t_pp"]
    # decode roofline over the whole token (B(p) = weights read per token + KV at the mean
    # position; token_embd is a 1-row gather, not streamed, so it is excluded)
    import refharness as R
    embd_bytes = R.row_bytes(types[0], hp["n_embd"]) * hp["n_vocab"]
    kv_bytes = 2 * hp["n_layer"] * hp["n_head_kv"] * (hp["n_embd"] // hp["n_head"]) * 2 * (n_past - steps / 2)
    token_gbs = (wb - embd_bytes + kv_bytes) / (ms_step * 1e-3) / 1e9
    # prefill roofline: F(n) = 2 * (layer weight elements) * n + attention 2 * 2 * n_head * D
    # * n(n+1)/2 per layer (causal QK^T and PV) + the output head once (only the last logits are computed)
    shapes = R.weight_shapes(hp)
    layer_elems = sum(k * n for i, (k, n) in enumerate(shapes) if i >= 3 and n > 1)
    n = args.prompt
    attn_flops = 4 * hp["n_layer"] * hp["n_embd"] * n * (n + 1) / 2
    pre_flops = 2 * layer_elems * n + attn_flops + 2 * hp["n_embd"] * hp["n_vocab"]
    pre_tflops = pre_flops / t_pp / 1e12
    roof = measure_roofline(K, torch)
    out = {
        "metric": "decode tok/s (Llama-3-8B Q4_K_M, 4k ctx); prefill tok/s in prefill_tok_s",
        "value": round(dec, 2), "unit": "tok/s", "n_gpus": n_dev, "steps": steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "q4_K/q6_K weights x q8_K activations (int8 dot, f32 accum); f16 KV", "data": "synthetic",
        "config": {"workload": "llama3-8b-q4_k_m ctx4096: prefill %d (ubatch %d) + greedy decode" % (args.prompt, args.ubatch),
                   "model": "Llama-3-8B-shape Q4_K_M random-init", "n_layer": hp["n_layer"],
                   "prompt_tokens": args.prompt, "gen_positions": [args.prompt + args.warmup, n_past],
                   "parallelism": par},
        "prefill_tok_s": round(pre, 1), "prefill_s": round(t_pp, 4),
        "decode_effective_GBps": round(token_gbs, 1), "decode_hbm_frac": round(token_gbs / HBM_PEAK_GBS, 4),   # one stage streams at a time
        "decode_bytes_per_token": int(wb - embd_bytes + kv_bytes),
        "weight_bytes_resident": wb,
        "roofline": roof,
        "prefill_roofline": {"bound": "mfma", "achieved": round(pre_tflops, 1), "peak": MFMA_F16_PEAK_TFLOPS * n_dev,
                             "unit": "TFLOP/s", "frac": round(pre_tflops / MFMA_F16_PEAK_TFLOPS / n_dev, 4),
                             # the Q4_K / Q5_K GEMMs run v_mfma_i32_32x32x32_i8 (2x the f16 rate per clock,
                             # MI355X_MICROARCH.md: Matrix cores), so against that peak the same work is half the fraction
                             "peak_i8": MFMA_I8_PEAK_TOPS * n_dev,
                             "frac_i8": round(pre_tflops / MFMA_I8_PEAK_TOPS / n_dev, 4),
                             "flops": int(pre_flops), "scope": "whole prefill (all kernels), F(n) of SURVEY.md 8d; "
                                                               "peak = %d GPU(s); frac vs the dense f16 peak, frac_i8 "
                                                               "vs the dense i8 peak" % n_dev},
    }
    if n_dev == 1 and not args.no_generate_path:
        try:
            out["generate_path"] = generate_path(hp, types, args.prompt, 256, args.ubatch)
        except Exception as e:  # reported, never fatal for the GPU number
            out["generate_path"] = {"error": str(e)[:300]}
    if not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(hp, types, args.cpu_threads)
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"error": str(e)[:300]}
    return out


if __name__ == "__main__":
    main()
