#!/bin/bash
# round-5: SQ / TCC counter passes over single GEMM shapes (tools/gemm_bench), per kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=3d-speaker_amd/lib/libspk_hip.so
P1=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_WAIT_INST_LDS,SQ_INSTS_SALU
P2=SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_ANY,SQ_INSTS_VMEM_RD,SQ_LDS_BANK_CONFLICT
P3=SQ_WAVE_CYCLES,SQ_LDS_IDX_ACTIVE,GRBM_GUI_ACTIVE,TCC_HIT_sum,TCC_MISS_sum
for sh in ${SHAPES:-l3_ds l4.convs0 l3.convs0 l3.conv1}; do
  i=0
  for p in $P1 $P2 $P3; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $p -d gpurun_out/sq_${sh}_$i -o run --output-format csv -- \
        ./tools/gemm_bench --reps 3 --shapes $sh $L > gpurun_out/sq_${sh}_$i.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "pass $i $sh rc=$rc"; tail -5 gpurun_out/sq_${sh}_$i.log; exit $rc; fi
    echo "== $sh pass $i"; python tools/pmc_sq.py gpurun_out/sq_${sh}_$i conv_gemm | head -3
  done
done
