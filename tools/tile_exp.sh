#!/bin/bash
# Per-step profiles of one arch under each x3 tile override (SPK_X3_TILE).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
arch=${1:-eres2netv2}
for t in default ${TILES:-128x128w4 128x128 256x128}; do
  echo "== tile $t $(date +%T)"
  if [ $t = default ]; then unset SPK_X3_TILE; else export SPK_X3_TILE=$t; fi
  timeout -k 10 300 python tools/profile_steps.py --arch $arch --json gpurun_out/tile_$t.json > gpurun_out/tile_$t.txt 2>&1 || exit $?
  head -1 gpurun_out/tile_$t.txt
  python tools/agg_steps.py gpurun_out/tile_$t.json | head -${ROWS:-18}
done
