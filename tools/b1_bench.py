"""Decode tok/s of the Llama-3-8B Q4_K_M graph driven through the ggml backend plugin (b1) by the REFERENCE host:
oracle/_ref/ref_b1 (the reference ggml library builds build_llama's graph every token, ggml_backend_sched splits it
over {our ROCm backend, the reference CPU backend}, our vtables dispatch every node) -- what a koboldcpp build that
links koboldcpp_hipblas.so as its GPU backend would get, as opposed to the expose ABI's fused runtime (bench.py).
A diagnostic: nothing here enters bench.py.

  python3 tools/b1_bench.py [n_layer] [n_past] [steps]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    nl = sys.argv[1] if len(sys.argv) > 1 else "32"
    npast = sys.argv[2] if len(sys.argv) > 2 else "3840"
    steps = sys.argv[3] if len(sys.argv) > 3 else "32"
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_b1")
    so = os.path.join(ROOT, "koboldcpp_amd", "koboldcpp_hipblas.so")
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "16"))
    r = subprocess.run([exe, so, nl, npast, steps], env=env, capture_output=True, text=True, timeout=900)
    sys.stderr.write(r.stderr[-2000:])
    print(r.stdout.strip(), flush=True)
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
