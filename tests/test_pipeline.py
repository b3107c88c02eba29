"""Layer-split pipeline (koboldcpp_amd/pipeline.py): layer placement vs the reference rule
(src/llama.cpp:7000-7036), and the send/recv protocol at world_size 2 and 3 over gloo on CPU with
a deterministic stand-in stage.  The GPU version of the same protocol (HipStage, both ranks on
one card, gloo transport) is in test_gpu_model.py::test_pipeline_two_stages_gloo."""
import bisect
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from koboldcpp_amd import pipeline as P


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


@pytest.mark.parametrize("n_layer,n_dev,ts", [
    (32, 1, [1]), (32, 2, [1, 1]), (32, 4, [1, 1, 1, 1]), (32, 8, [1] * 8), (80, 8, [1] * 8),
    (22, 3, [3, 1, 2]), (32, 2, [0.3, 0.7]),
])
def test_assign_layers_matches_reference_rule(n_layer, n_dev, ts):
    dev, out = P.assign_layers(n_layer, n_dev, ts)
    rdev, rout = ref_assign(n_layer, n_dev, ts, n_layer + 1)
    assert dev == rdev and out == rout
    ranges = P.stage_ranges(n_layer, n_dev, ts)
    assert ranges[0][0] == 0 and ranges[-1][1] == n_layer
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))


def test_stage_ranges_8b_on_8():
    # 33 "GPU layers" over 8 equal devices: 5,4,4,4,4,4,4,3 repeating layers; output on the last
    r = P.stage_ranges(32, 8)
    assert [b - a for a, b in r] == [5, 4, 4, 4, 4, 4, 4, 3]


E, V = 8, 97


class ToyStage:
    """Deterministic stand-in with the HipStage interface: residual stream h[T][E] (float64 math
    on float32 storage), layer l: h = tanh(0.9 h + 0.01 (l+1) + 0.001 pos)."""

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

    def hidden_to(self, buf, T, on_device):
        buf[:T * E].copy_(torch.from_numpy(self.h[:T].reshape(-1).copy()))

    def hidden_from(self, buf, T, on_device):
        self.h[:T] = buf[:T * E].numpy().reshape(T, E)

    def stream_ptr(self):
        return None


def run_sequence(pipe_decode, prompt, n_gen):
    toks = []
    tok = pipe_decode(prompt, len(prompt), 0)
    toks.append(tok)
    n_past = len(prompt)
    for _ in range(n_gen):
        tok = pipe_decode([tok] if tok is not None else None, 1, n_past)
        toks.append(tok)
        n_past += 1
    return toks


def single_stage_tokens(n_layer, prompt, n_gen, ub):
    st = ToyStage(0, n_layer, True, True, ub)

    def dec(tokens, T, n_past):
        for i in range(0, T, ub):
            t = min(ub, T - i)
            st.run(tokens[i:i + t], t, n_past + i)
        return st.argmax()
    return run_sequence(dec, prompt, n_gen)


def _worker(rank, world, port, n_layer, prompt, n_gen, ub, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        il0, il1 = P.stage_ranges(n_layer, world)[rank]
        st = ToyStage(il0, il1, rank == 0, rank == world - 1, ub)
        pipe = P.Pipeline.__new__(P.Pipeline)
        # the real constructor, minus the CUDA stream (host transport)
        P.Pipeline.__init__(pipe, st, rank, world, E, ub, device_comm=False)

        def dec(tokens, T, n_past):
            return pipe.decode(tokens if rank == 0 else None, T, n_past)
        toks = run_sequence(dec, prompt, n_gen)
        pipe.flush()
        q.put((rank, toks))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_pipeline_protocol_gloo(world):
    n_layer, ub, n_gen = 7, 4, 5
    prompt = [3, 14, 15, 92, 65, 35, 89, 79, 32, 38]          # 10 tokens -> ubatches 4,4,2
    want = single_stage_tokens(n_layer, prompt, n_gen, ub)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_layer, prompt, n_gen, ub, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == want                      # rank 0 sees every greedy token
    assert got[world - 1] == want
