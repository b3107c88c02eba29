"""Diagnostics: the drop-in generate() leg alone (bench.py generate_path on the Llama-3-8B Q4_K_M bench model, 256-token
prompt, N greedy tokens), for rocprofv3 --kernel-trace: the gaps between consecutive decode steps show what the host
loop of generate() costs beside the device-greedy loop."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
hp = dict(bench.LLAMA3_8B)
t0 = time.perf_counter()
r = bench.generate_path(hp, bench.q4_k_m_types(32), 256, n, 512)
print(r, "wall %.2f s" % (time.perf_counter() - t0))
