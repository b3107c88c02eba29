"""Stage hand-off cost on one GPU (verdict r05 item 2): the Llama-3-8B bench model through the drop-in engine
(kcpp_engine_bench) as 1 stage and as N virtual stages (KCPP_VIRTUAL_DEVICES), printing ms per token and the
per-hop cost.  Run under `rocprofv3 --kernel-trace --hip-trace` to see where each hop's time goes
(tools/handoff_gaps.py reads the traces).

  python3 tools/handoff_trace.py [N_STAGES] [STEPS]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))

import koboldcpp_amd.lib as K  # noqa: E402
import refharness as R  # noqa: E402

LLAMA3_8B = dict(n_vocab=128256, n_embd=4096, n_head=32, n_head_kv=8, n_layer=32, n_ff=14336, n_ctx=4096,
                 eps=1e-5, rope_base=500000.0)


def main():
    ns = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    types = R.q4_k_m_types(32)
    os.environ["KCPP_VIRTUAL_DEVICES"] = "1"
    out = {}
    for n in (1, ns):
        t0 = time.perf_counter()
        r = K.engine_bench(LLAMA3_8B, types, n, 512, 512, 8, steps)
        out[n] = r
        print("stages %d: %.4f ms/token (prefill %.1f ms) wall %.1f s" % (n, r["decode_s"] / steps * 1e3,
                                                                        r["prefill_s"] * 1e3, time.perf_counter() - t0),
              flush=True)
    hop = (out[ns]["decode_s"] - out[1]["decode_s"]) / steps / ns * 1e6
    print(json.dumps({"per_hop_us": round(hop, 2), "stages": ns, "steps": steps,
                      "one_ms": round(out[1]["decode_s"] / steps * 1e3, 4),
                      "n_ms": round(out[ns]["decode_s"] / steps * 1e3, 4)}), flush=True)


if __name__ == "__main__":
    main()
