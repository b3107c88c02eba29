"""The multi-GPU layer-split path of the drop-in engine (koboldcpp_amd/csrc/expose.cpp: build_stages / forward /
greedy_step over HipOps), checked on CPU:

* layer placement (load_model's split_layers, through the kcpp_split_layers hook) against a direct restatement of
  the reference rule (src/llama.cpp:7000-7036);
* the schedule's enqueue order (kcpp_pipeline_trace: the same forward() / greedy_step() code over the trace
  backend): ubatches pipelined stage to stage, every hand-off before its consumer, the greedy token going home to
  stage 0 on the device with no host step in between;
* the schedule EXECUTED by world_size 2 and 3 gloo process groups, one process per stage with a deterministic
  stand-in stage: each rank plays its part of the shipped trace (decodes, hand-off send / recv, the token home) and
  the greedy tokens equal a single stage's.  The GPU runs of the same engine are in test_gpu_expose.py
  (test_generate_layer_split_pipeline_matches_single_stage, test_engine_bench_layer_split)."""
import bisect
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import koboldcpp_amd.lib as K


def ref_assign(n_layer, n_dev, ts, n_gpu_layers):
    # direct restatement of src/llama.cpp:7010-7036 in float32 arithmetic
    sp, acc = [], np.float32(0)
    for v in ts:
        acc = np.float32(acc + np.float32(v))
        sp.append(acc)
    sp = [np.float32(x / acc) for x in sp]
    act = min(n_gpu_layers, n_layer + 1)
    dev = [bisect.bisect_right(sp, np.float32(i) / np.float32(act)) for i in range(n_layer)]
    out = bisect.bisect_right(sp, np.float32(act - 1) / np.float32(act))
    return dev, out


def stage_ranges(n_layer, n_dev, ts=None):
    dev, _ = K.split_layers(n_layer, n_dev, ts)
    out, i = [], 0
    while i < n_layer:
        j = i
        while j < n_layer and dev[j] == dev[i]:
            j += 1
        out.append((i, j))
        i = j
    return out


@pytest.mark.parametrize("n_layer,n_dev,ts", [
    (32, 1, [1]), (32, 2, [1, 1]), (32, 4, [1, 1, 1, 1]), (32, 8, [1] * 8), (80, 8, [1] * 8),
    (22, 3, [3, 1, 2]), (32, 2, [0.3, 0.7]),
])
def test_split_layers_matches_reference_rule(n_layer, n_dev, ts):
    dev, out = K.split_layers(n_layer, n_dev, ts)
    rdev, rout = ref_assign(n_layer, n_dev, ts, n_layer + 1)
    assert dev == rdev and out == rout
    ranges = stage_ranges(n_layer, n_dev, ts)
    assert ranges[0][0] == 0 and ranges[-1][1] == n_layer
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))


def test_stage_ranges_8b_on_8():
    # 33 "GPU layers" over 8 equal devices: 5,4,4,4,4,4,4,3 repeating layers; output on the last
    assert [b - a for a, b in stage_ranges(32, 8)] == [5, 4, 4, 4, 4, 4, 4, 3]


def test_schedule_single_stage():
    tr = K.pipeline_trace(1, 512, 1000, 0, 2)
    assert tr == ["d0:512@0", "d0:488@512", "a", "k", "s0@1000", "k", "s0@1001", "k"]


@pytest.mark.parametrize("S", [2, 3, 8])
def test_schedule_stages(S):
    T, ub, n0, steps = 10, 4, 7, 3
    tr = K.pipeline_trace(S, ub, T, n0, steps)
    want = []
    for i, t in ((0, 4), (4, 4), (8, 2)):            # ubatches of the prefill, each through every stage
        for s in range(S):
            if s:
                want.append("h%d:%d" % (s, t))
            want.append("d%d:%d@%d" % (s, t, n0 + i))
    want += ["a", "k"]                                # the prefill's token home on device
    for j in range(steps):                            # greedy steps: token in, hand-offs, token home
        for s in range(S):
            if s:
                want.append("h%d:1" % s)
            want.append("s%d@%d" % (s, n0 + T + j))
        want.append("k")
    assert tr == want


# ---------------------------------------------------------------- the schedule executed over gloo
E, V = 8, 97


class ToyStage:
    """Deterministic stand-in stage: residual stream h[T][E] (float64 math on float32 storage), layer l:
    h = tanh(0.9 h + 0.01 (l+1) + 0.001 pos); the embedding stage maps ids to sin(tok * k)."""

    def __init__(self, il0, il1, first, last, ub):
        self.il0, self.il1, self.first, self.last, self.ub = il0, il1, first, last, ub
        self.h = np.zeros((ub, E), np.float32)
        self.T = 0

    def run(self, tokens, T, n_past):
        if self.first:
            tok = np.asarray(tokens, np.float64)
            self.h[:T] = (np.sin(tok[:, None] * np.arange(1, E + 1)[None, :])).astype(np.float32)
        pos = n_past + np.arange(T)[:, None]
        for l in range(self.il0, self.il1):
            self.h[:T] = np.tanh(0.9 * self.h[:T] + 0.01 * (l + 1) + 0.001 * pos).astype(np.float32)
        self.T = T

    def argmax(self):
        return int(np.floor(np.abs(self.h[self.T - 1]).sum() * 1000)) % V


def single_stage_tokens(n_layer, prompt, n_gen, ub):
    st = ToyStage(0, n_layer, True, True, ub)
    for i in range(0, len(prompt), ub):
        st.run(prompt[i:i + ub], min(ub, len(prompt) - i), i)
    toks = [st.argmax()]
    for j in range(n_gen):
        st.run([toks[-1]], 1, len(prompt) + j)
        toks.append(st.argmax())
    return toks


def play(rank, world, st, trace, prompt):
    """this rank's part of the engine's schedule: stage `rank`'s decodes and steps, its side of each hand-off and
    of the token's way home (gloo send / recv standing in for RCCL / xGMI peer copies)"""
    last = world - 1
    cursor, tok, toks = 0, None, []
    for op in trace:
        if op[0] == "d":                            # d<s>:<t>@<n_past>
            s, rest = op[1:].split(":")
            t, n_past = (int(v) for v in rest.split("@"))
            if int(s) == rank:
                st.run(prompt[cursor:cursor + t] if rank == 0 else None, t, n_past)
                cursor += t
        elif op[0] == "h":                          # h<s>:<t>: stage s-1's residual stream -> stage s
            s, t = (int(v) for v in op[1:].split(":"))
            if rank == s - 1:
                dist.send(torch.from_numpy(st.h[:t].copy()), dst=s)
            elif rank == s:
                buf = torch.empty((t, E), dtype=torch.float32)
                dist.recv(buf, src=s - 1)
                st.h[:t] = buf.numpy()
        elif op[0] == "s":                          # s<s>@<n_past>: one token, input already on the stage
            s, n_past = (int(v) for v in op[1:].split("@"))
            if s == rank:
                st.run([tok] if rank == 0 else None, 1, n_past)
                if rank == last:
                    tok = st.argmax()
                    toks.append(tok)
        elif op == "a":
            if rank == last:
                tok = st.argmax()
                toks.append(tok)
        elif op == "k":                             # the last stage's token home to stage 0
            if world > 1 and rank in (0, last):
                t = torch.tensor([tok if rank == last else 0], dtype=torch.int64)
                if rank == last:
                    dist.send(t, dst=0)
                else:
                    dist.recv(t, src=last)
                    tok = int(t.item())
                    toks.append(tok)
    return toks


def _worker(rank, world, port, ranges, prompt, ub, trace, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        il0, il1 = ranges[rank]
        st = ToyStage(il0, il1, rank == 0, rank == world - 1, ub)
        q.put((rank, play(rank, world, st, trace, prompt)))
    except Exception as e:            # reported to the parent instead of a silent exit
        q.put((rank, "error: %r" % (e,)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_engine_schedule_gloo(world):
    n_layer, ub, n_gen = 7, 4, 5
    prompt = [3, 14, 15, 92, 65, 35, 89, 79, 32, 38]          # 10 tokens -> ubatches 4,4,2
    want = single_stage_tokens(n_layer, prompt, n_gen, ub)
    trace = K.pipeline_trace(world, ub, len(prompt), 0, n_gen)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ranges = stage_ranges(n_layer, world)        # the engine's placement (the workers need no native library)
    procs = [ctx.Process(target=_worker, args=(r, world, port, ranges, prompt, ub, trace, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=60) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[world - 1] == want               # the last stage computes every greedy token
    assert got[0] == want                       # and each one reaches stage 0 (the token home)
