cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for sh in l3_ds l3.conv1 l3.convs0; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pl_${sh}_$c -o run --output-format csv -- tools/gemm_bench --reps 3 --shapes $sh 3d-speaker_amd/lib/libspk_hip.so > gpurun_out/pl_${sh}_$c.log 2>&1 || exit 1
  done
  python tools/pmc_traffic.py gpurun_out/pl_${sh}_FETCH_SIZE gpurun_out/pl_${sh}_WRITE_SIZE -o gpurun_out/pl_${sh}.json > gpurun_out/pl_${sh}.txt 2>&1; echo "$sh: $(head -3 gpurun_out/pl_${sh}.txt)"
done
