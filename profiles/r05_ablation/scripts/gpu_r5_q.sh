#!/bin/bash
# round-5 GPU pass Q: PMC HBM traffic per launch of single layers (tools/gemm_bench one shape per
# run, so each kernel name in the counter files is that layer alone): layer3_ds, l3.conv1, l3.convs0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=3d-speaker_amd/lib/libspk_hip.so
for s in l3_ds l3.conv1 l3.convs0; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmcl_${s}_$c -o run --output-format csv -- \
      ./tools/gemm_bench --reps 3 --shapes $s $L > gpurun_out/pmcl_${s}_$c.log 2>&1 || { tail -5 gpurun_out/pmcl_${s}_$c.log; exit 1; }
  done
  python tools/pmc_traffic.py gpurun_out/pmcl_${s}_FETCH_SIZE gpurun_out/pmcl_${s}_WRITE_SIZE -o gpurun_out/pmcl_$s.json > gpurun_out/pmcl_$s.txt 2>&1
  echo "== $s"; grep -v split_f16 gpurun_out/pmcl_$s.txt | head -4
done
