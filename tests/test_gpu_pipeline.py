"""Layer-split pipeline on the GPU: two stage processes sharing the one card of the test box,
hidden state handed over with the host-staged gloo transport (RCCL p2p needs two devices; the
driver's multi-GPU bench exercises it).  The split model must produce exactly the tokens and the
final hidden state of the unsplit model: same kernels, same order, only the stage boundary moves."""
import os
import socket

import numpy as np
import pytest

import refharness as R

pytestmark = pytest.mark.gpu

HP = dict(R.TINY, n_layer=4)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tokens_fn, prompt, n_gen):
    toks = [tokens_fn(prompt, len(prompt), 0)]
    n = len(prompt)
    for _ in range(n_gen):
        toks.append(tokens_fn([toks[-1]] if toks[-1] is not None else None, 1, n))
        n += 1
    return toks


def _worker(rank, world, port, prompt, n_gen, ub, q):
    import torch
    import torch.distributed as dist
    from koboldcpp_amd import pipeline as P
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        il0, il1 = P.stage_ranges(HP["n_layer"], world)[rank]
        types = R.q4_k_m_types(HP["n_layer"])
        st = P.HipStage(HP, types, 0, il0, il1, rank == 0, rank == world - 1, ub, seed=1234)
        pipe = P.Pipeline(st, rank, world, HP["n_embd"], ub, device_comm=False)
        toks = _run(lambda t, T, n: pipe.decode(t if rank == 0 else None, T, n), prompt, n_gen)
        pipe.flush()
        hid = st.m.read_hidden(HP["n_embd"]) if rank == world - 1 else None
        st.close()
        q.put((rank, toks, hid))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_pipeline_stages_gloo(world):
    import torch.multiprocessing as mp
    import koboldcpp_amd.lib as K
    ub, n_gen = 16, 6
    prompt = [(7 * i + 3) % HP["n_vocab"] for i in range(40)]      # 3 ubatches: 16, 16, 8
    m = K.Model(HP, R.q4_k_m_types(HP["n_layer"]), max_ubatch=ub)
    m.synth(1234)

    def single(t, T, n):
        m.decode(t, n, want_logits=False)
        return m.argmax()
    want = _run(single, prompt, n_gen)
    want_h = m.read_hidden(HP["n_embd"])
    m.close()

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, prompt, n_gen, ub, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, toks, hid = q.get(timeout=300)
        got[r] = (toks, hid)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][0] == want
    assert got[world - 1][0] == want
    np.testing.assert_array_equal(got[world - 1][1], want_h)
