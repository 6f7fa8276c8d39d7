#!/bin/bash
# Session r4x: tiling sweep of the float stage-1 kernel on the 16-bit beam (HD_S1T_SG subbands
# per workgroup, HD_S1T_KB first LDS budget), ms per step.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --nbits 16 --steps 3 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 0"
for e in "" "HD_S1T_KB=156" "HD_S1T_SG=4" "HD_S1T_SG=4 HD_S1T_KB=96" "HD_S1T_SG=4 HD_S1T_KB=156" "HD_S1T_SG=2" "HD_S1T_SG=2 HD_S1T_KB=96"; do
  env $e timeout -k 10 300 $B > gpurun_out/abe.log 2>&1 || { echo "bench failed ($e)"; exit 1; }
  s=$(python3 scripts/benchline.py gpurun_out/abe.log) || { echo "no bench line ($e)"; exit 1; }
  echo "[$e] $s"
done
echo "r4x done"
