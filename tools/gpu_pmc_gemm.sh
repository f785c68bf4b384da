cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/${TAG:-r6o}_pmc$i -o run --output-format csv -- tools/gemm_bench --reps 3 --shapes l3.conv1,l3.conv3,l3.convs0,l3_ds ${LIB:-ablibs/libspk_cur.so} > gpurun_out/${TAG:-r6o}_pmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${TAG:-r6o}_pmc$i.log; exit 1; }
  python3 tools/pmc_sq.py gpurun_out/${TAG:-r6o}_pmc$i conv_gemm_x3f > gpurun_out/${TAG:-r6o}_pmc$i.txt 2>&1; cat gpurun_out/${TAG:-r6o}_pmc$i.txt
done
