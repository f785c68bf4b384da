#!/bin/bash
# round-5 GPU pass E: full GPU test suite + smoke + bench (checkpoint)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_gputest_e.log 2>&1 || { tail -30 gpurun_out/r5_gputest_e.log; exit 1; }
tail -2 gpurun_out/r5_gputest_e.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke_e.log 2>&1 || { tail -20 gpurun_out/r5_smoke_e.log; exit 1; }
tail -2 gpurun_out/r5_smoke_e.log
timeout -k 10 400 python bench.py > gpurun_out/r5_bench_e.json 2> gpurun_out/r5_bench_e.err || { tail -20 gpurun_out/r5_bench_e.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r5_bench_e.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['per_launch_roofline']['frac'])"
