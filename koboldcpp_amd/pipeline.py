"""Layer-split pipeline over several GPUs of one node: one process per GPU, hidden-state handoff
by point-to-point send/recv (RCCL over xGMI with backend "nccl"; host-staged with "gloo").

Reference behaviour this mirrors:
  * layer placement -- llm_load_tensors, LLAMA_SPLIT_MODE_LAYER (src/llama.cpp:7000-7036):
    cumulative, normalised tensor_split; layer i -> upper_bound(splits, i / act_gpu_layers);
    the output head on the device of act_gpu_layers - 1 (the last one for an even split);
  * inter-device copy of the residual stream at each split boundary -- ggml_backend_sched_compute_splits
    (ggml/src/ggml-backend.cpp:2108-2201) + ggml_backend_cuda_cpy_tensor_async
    (ggml/src/ggml-cuda.cu:2392-2445).  Here it is a send/recv of [T x n_embd] f32 per ubatch;
  * ubatch splitting -- llama_decode_internal (src/llama.cpp:17187-17201).  Stages work on
    different ubatches at the same time, so prefill pipelines across GPUs.

The embedding lives on rank 0 (the reference keeps it on the host, src/llama.cpp:6990: an
equivalent 16 KB gather either way).  The greedy token of the last stage is sent back to rank 0.

The stage is anything with the small interface below (HipStage wraps the native runtime); the
protocol is tested with world_size 2 on CPU (gloo) in tests/test_pipeline.py.
"""
import os
import time

import numpy as np


def split_points(tensor_split, n_dev):
    """cumulative normalised split points, float32 like the reference (src/llama.cpp:7012-7021)"""
    ts = list(tensor_split) if tensor_split is not None else []
    ts = (ts + [0.0] * n_dev)[:n_dev]
    if all(x == 0.0 for x in ts):
        ts = [1.0] * n_dev                 # reference: free memory per device; equal devices here
    sp = np.zeros(n_dev, np.float32)
    acc = np.float32(0.0)
    for i, v in enumerate(ts):
        acc = np.float32(acc + np.float32(v))
        sp[i] = acc
    return (sp / acc).astype(np.float32)


def assign_layers(n_layer, n_dev, tensor_split=None, n_gpu_layers=None):
    """device of every repeating layer and of the output head (src/llama.cpp:7023-7036)"""
    n_gpu_layers = n_layer + 1 if n_gpu_layers is None else n_gpu_layers
    if n_gpu_layers <= n_layer:
        raise ValueError("partial offload (CPU layers) is out of scope: n_gpu_layers must exceed n_layer")
    sp = split_points(tensor_split, n_dev)
    act = min(n_gpu_layers, n_layer + 1)
    dev = [int(np.searchsorted(sp, np.float32(i) / np.float32(act), side="right")) for i in range(n_layer)]
    out = int(np.searchsorted(sp, np.float32(act - 1) / np.float32(act), side="right"))
    return [min(d, n_dev - 1) for d in dev], min(out, n_dev - 1)


def stage_ranges(n_layer, n_dev, tensor_split=None):
    """[(il0, il1)] per device; the layer assignment must be monotone (it is, for cumulative splits)"""
    dev, out = assign_layers(n_layer, n_dev, tensor_split)
    if out != n_dev - 1:
        raise ValueError("output head must live on the last stage (got device %d)" % out)
    ranges = []
    for d in range(n_dev):
        ids = [i for i, x in enumerate(dev) if x == d]
        if ids:
            if ids != list(range(ids[0], ids[-1] + 1)):
                raise ValueError("non-contiguous layer assignment")
            ranges.append((ids[0], ids[-1] + 1))
        else:
            ranges.append((ranges[-1][1] if ranges else 0,) * 2)
    return ranges


class HipStage:
    """One pipeline stage on the local GPU (koboldcpp_amd.lib.Model over layers [il0, il1))."""

    def __init__(self, hp, types, device, il0, il1, first, last, max_ubatch=512, seed=None):
        from . import lib as K
        self.hp, self.first, self.last, self.ub = dict(hp), first, last, max_ubatch
        self.m = K.Model(hp, types, device=device, il0=il0, il1=il1, has_embed=first, has_output=last,
                         max_ubatch=max_ubatch)
        if seed is not None:
            self.m.synth(seed)

    def run(self, tokens, T, n_past):
        """enqueue the stage's layers for T tokens.  Prefill ubatches (T > 1, n_past passed by value) are only
        enqueued, so a rank works on ubatch u + 1 while the next rank works on u; single-token steps read their
        position from the stage's pinned word inside the replayed graph and stay synchronous, so the host can
        never rewrite that word under a pending replay"""
        tok = tokens if self.first else None
        if T > 1:
            self.m.decode_async(tok, n_past, n_tokens=T)
        else:
            self.m.decode(tok, n_past, want_logits=False, n_tokens=T)

    def argmax(self):
        return self.m.argmax()

    def hidden_to(self, buf, T, on_device):
        """copy the stage output [T][n_embd] into buf (torch tensor); synchronous for host buffers"""
        self.m.hidden_io(buf.data_ptr(), T * self.hp["n_embd"], 0, to_buf=True)
        if not on_device:
            self.m.sync()

    def hidden_from(self, buf, T, on_device):
        self.m.hidden_io(buf.data_ptr(), T * self.hp["n_embd"], 0, to_buf=False)
        if not on_device:
            self.m.sync()

    def stream_ptr(self):
        return self.m.stream()

    def close(self):
        self.m.close()


class Pipeline:
    """Drives one stage per rank.  decode() is collective: every rank calls it with the same
    (T, n_past); rank 0 passes the token ids.  Returns the greedy next token on rank 0 and on the
    last rank (None elsewhere)."""

    def __init__(self, stage, rank, world, n_embd, max_ubatch, device_comm):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.stage, self.rank, self.world, self.E, self.ub = stage, rank, world, n_embd, max_ubatch
        self.on_dev = device_comm                   # nccl: device buffers; gloo: host buffers
        dev = torch.device("cuda", torch.cuda.current_device()) if device_comm else torch.device("cpu")
        # separate receive and (double-buffered) send buffers: a middle stage receives ubatch u+1
        # while its send of ubatch u may still be in flight
        self.rbuf = torch.empty(max_ubatch * n_embd, dtype=torch.float32, device=dev)
        self.sbufs = [torch.empty(max_ubatch * n_embd, dtype=torch.float32, device=dev) for _ in range(2)]
        self.tok = torch.zeros(1, dtype=torch.int32, device=dev)
        self._pend = [None, None]
        self._ext = None
        if device_comm:
            # RCCL work is ordered against the stage's own HIP stream
            self._ext = torch.cuda.ExternalStream(stage.stream_ptr())

    def _ctx(self):
        import contextlib
        return self.torch.cuda.stream(self._ext) if self._ext is not None else contextlib.nullcontext()

    def _send(self, slot, T, dst):
        if self._pend[slot] is not None:          # the buffer is still being sent (two ubatches back)
            with self._ctx():                     # order the stage stream after that send
                self._pend[slot].wait()
        buf = self.sbufs[slot]
        self.stage.hidden_to(buf, T, self.on_dev)
        with self._ctx():
            self._pend[slot] = self.dist.isend(buf[:T * self.E], dst)

    def _recv(self, T, src):
        buf = self.rbuf
        with self._ctx():
            self.dist.recv(buf[:T * self.E], src)
        self.stage.hidden_from(buf, T, self.on_dev)

    def flush(self):
        for i, w in enumerate(self._pend):
            if w is not None:
                with self._ctx():
                    w.wait()
                self._pend[i] = None

    def decode(self, tokens, T, n_past):
        r, W = self.rank, self.world
        nub = (T + self.ub - 1) // self.ub
        for u in range(nub):
            i0 = u * self.ub
            t = min(self.ub, T - i0)
            if r > 0:
                self._recv(t, r - 1)
            self.stage.run(tokens[i0:i0 + t] if (r == 0 and tokens is not None) else None, t, n_past + i0)
            if r < W - 1:
                self._send(u & 1, t, r + 1)
        tok = None
        if r == W - 1:
            tok = self.stage.argmax()
            if W > 1:
                with self._ctx():                 # fill, send and read back all on the stage stream
                    self.tok.fill_(tok)
                    self.dist.send(self.tok, 0)
        elif r == 0:
            with self._ctx():
                self.dist.recv(self.tok, W - 1)
                tok = int(self.tok.item())
        return tok


def bench_main(args, world, rank, local):
    """bench.py for N > 1 (torchrun): Llama-3-8B Q4_K_M split over `world` GPUs by layers."""
    import json
    import torch
    import torch.distributed as dist
    import bench as B

    backend = os.environ.get("KCPP_PIPE_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if local >= ndev:
        # rehearsal on fewer GPUs than ranks (host-staged gloo transport only; RCCL needs distinct GPUs)
        if os.environ.get("KCPP_PIPE_SHARE_GPU") != "1" or backend == "nccl":
            raise RuntimeError("local rank %d but only %d GPU(s) visible" % (local, ndev))
        local = local % ndev
    torch.cuda.set_device(local)
    dist.init_process_group(backend=backend, init_method="env://", world_size=world, rank=rank)
    hp = dict(B.LLAMA3_8B)
    if args.layers:
        hp["n_layer"] = args.layers
    types = B.q4_k_m_types(hp["n_layer"])
    ranges = stage_ranges(hp["n_layer"], world)
    il0, il1 = ranges[rank]
    stage = HipStage(hp, types, local, il0, il1, rank == 0, rank == world - 1, args.ubatch, seed=1234)
    pipe = Pipeline(stage, rank, world, hp["n_embd"], args.ubatch, device_comm=(backend == "nccl"))
    dev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")

    def barrier_sync():
        dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    prompt = [16 + (i % 2) for i in range(args.prompt)]
    pipe.decode(prompt[:64], 64, 0)                       # warm-up (first touch, comm setup)
    pipe.flush()
    barrier_sync()
    t0 = time.perf_counter()
    tok = pipe.decode(prompt, len(prompt), 0)
    pipe.flush()
    torch.cuda.synchronize()
    t_pp = max_over_ranks(time.perf_counter() - t0)
    barrier_sync()
    n_past = len(prompt)
    for _ in range(args.warmup):
        tok = pipe.decode([tok] if rank == 0 else None, 1, n_past)
        n_past += 1
    steps = min(args.steps, hp["n_ctx"] - n_past)
    pipe.flush()
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        tok = pipe.decode([tok] if rank == 0 else None, 1, n_past)
        n_past += 1
    pipe.flush()
    torch.cuda.synchronize()
    t_tg = max_over_ranks(time.perf_counter() - t0)
    barrier_sync()
    wb = max_over_ranks(float(stage.m.weight_bytes()))
    from . import lib as K
    roof = B.measure_roofline(K, torch) if rank == 0 else None
    stage.close()
    if rank == 0:
        dec = steps / t_tg
        out = {
            "metric": "decode tok/s (Llama-3-8B Q4_K_M, 4k ctx); prefill tok/s in prefill_tok_s",
            "value": round(dec, 2), "unit": "tok/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
            "ms_per_step": round(t_tg / steps * 1e3, 4), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None,
            "dtype": "q4_K/q6_K weights x q8_K activations (int8 dot, f32 accum); f16 KV", "data": "synthetic",
            "config": {"workload": "llama3-8b-q4_k_m ctx4096: prefill %d (ubatch %d) + greedy decode, layer split"
                                   % (args.prompt, args.ubatch),
                       "model": "Llama-3-8B-shape Q4_K_M random-init", "n_layer": hp["n_layer"],
                       "prompt_tokens": args.prompt, "parallelism": "pipeline (layer split) x%d, %s p2p" % (world, backend),
                       "stage_layers": ranges},
            "prefill_tok_s": round(args.prompt / t_pp, 1), "prefill_s": round(t_pp, 4),
            "max_stage_weight_bytes": int(wb),
            "roofline": roof,
            "cpu_baseline": None,
        }
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()
