# down-projection variants (tools only)
for c in "down q4k pro2" "down q4k pro0" "glu q4k pro1" "wo q4k pro0" "qkv q4k pro1 rope"; do
  for v in 0 2; do
    KCPP_Q4K_DOWN=$v PROBE_CASE="$c" timeout -k 10 120 python tools/stream_probe.py dec | sed "s/^/v=$v /" || exit 1
  done
done
