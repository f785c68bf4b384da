#!/bin/bash
# Diagnostics: SQ counter passes over one ERes2NetV2 forward + small-batch step profiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/list_avail.txt 2>&1 || true
P1=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_WAIT_INST_LDS,SQ_INSTS_SALU
P2=SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_ANY,SQ_INSTS_VMEM_RD,SQ_LDS_BANK_CONFLICT
i=0
for p in $P1 $P2; do
  i=$((i+1))
  echo "== pmc pass $i $(date +%T)"
  timeout -s KILL 120 rocprofv3 --pmc $p -d gpurun_out/sq$i -o run --output-format csv -- \
      python tools/profile_steps.py --arch eres2netv2 > gpurun_out/sq$i.log 2>&1
  rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/sq$i.log; exit $rc; fi
  python tools/pmc_sq.py gpurun_out/sq$i | head -12
done
for b in 8 16 32; do
  echo "== steps B=$b $(date +%T)"
  timeout -k 10 200 python tools/profile_steps.py --arch eres2netv2 --batch $b --json gpurun_out/steps_b$b.json > gpurun_out/steps_b$b.txt 2>&1 || exit $?
  head -1 gpurun_out/steps_b$b.txt
done
timeout -k 10 200 python tools/profile_steps.py --arch eres2netv2 --json gpurun_out/steps_b256.json > gpurun_out/steps_b256.txt 2>&1
head -1 gpurun_out/steps_b256.txt
