#!/bin/bash
# Round 4: where the LDS-DMA ring GEMM's time goes -- per-step timings of ERes2NetV2 with the
# ring (persistent, and one block per tile), its ablation builds (tools/ring_exp.sh: r1 no MFMA,
# r2 no in-loop DMA, r3 no epilogue stores, r5 = 1+2+3) and the register-staged GEMM.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=3d-speaker_amd/lib/libspk_hip.so
LIBS="$L $L:SPK_RING=1 $L:SPK_RING=1,SPK_RING_GRID=0 ab/libspk_r1.so:SPK_RING=1 ab/libspk_r2.so:SPK_RING=1 ab/libspk_r3.so:SPK_RING=1 ab/libspk_r5.so:SPK_RING=1" \
  REPS=1 ARCHS=eres2netv2 bash tools/gpu_ab.sh
