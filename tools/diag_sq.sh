#!/bin/bash
# Diagnostics: SQ counter passes over one ERes2NetV2 forward, or over SQ_CMD (a python script
# and its arguments); per-kernel ratios to SQ_WAVE_CYCLES.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P1=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_WAIT_INST_LDS,SQ_INSTS_SALU
P2=SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_ANY,SQ_INSTS_VMEM_RD,SQ_LDS_BANK_CONFLICT
P3=SQ_WAVE_CYCLES,SQ_INSTS_VMEM_WR,SQ_ACTIVE_INST_MISC,SQ_ACTIVE_INST_FLAT,SQ_INST_CYCLES_VMEM_RD,SQ_WAVES,SQ_LDS_IDX_ACTIVE,SQ_ACTIVE_INST_SCA
i=0
for p in $P1 $P2 $P3; do
  i=$((i+1))
  echo "== pmc pass $i $(date +%T)"
  timeout -s KILL 120 rocprofv3 --pmc $p -d gpurun_out/sq$i -o run --output-format csv -- \
      python ${SQ_CMD:-tools/profile_steps.py --arch ${ARCH:-eres2netv2}} > gpurun_out/sq$i.log 2>&1
  rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/sq$i.log; exit $rc; fi
  python tools/pmc_sq.py gpurun_out/sq$i | head -8
done
