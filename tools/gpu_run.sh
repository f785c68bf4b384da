#!/bin/bash
# GPU passes of a round (one script, PHASE selects; every GPU step under its own time limit,
# the script stops at the first fatal status):
#   PHASE=tests  TESTS="tests/x.py ..."   pytest -m gpu on the named files (default: all)
#   PHASE=bench                            smoke + bench (20 steps)
#   PHASE=steps  ARCHS="eres2netv2 ..."    per-step HIP-event profiles
#   PHASE=gemm   LIBS="a.so b.so" SHAPES=..  tools/gemm_bench A/B of library builds
#   PHASE=ab     LIBS="a.so b.so" ARCHS=..   per-step profiles of several builds (SPK_HIP_LIB)
#   PHASE=core                             smoke, pytest -m gpu, steps, PMC (FETCH/WRITE, SQ),
#                                          rocprofv3 --kernel-trace --stats, bench
#   PHASE=workloads                        C1 / C3 / C3 fp16 / models / C4 / C5
# Outputs under gpurun_out/ (TAG prefixes the file names).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r6}
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
phase() { case " ${PHASE:-core} " in *" $1 "*) return 0;; *) return 1;; esac; }
rc=0

if phase smoke || phase core || phase bench; then
  echo "== smoke $(date +%T)"
  timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if phase tests || phase core; then
  echo "== pytest -m gpu ${TESTS:-tests} $(date +%T)"
  timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -v -rf --timeout 300 --timeout-method thread \
      > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}_pytest_gpu.log | tail -${NTAIL:-12}
  tail -2 gpurun_out/${TAG}_pytest_gpu.log
  if fatal $rc; then exit $rc; fi
fi
if phase gemm; then
  [ tools/gemm_bench -nt 3d-speaker_amd/csrc/common.h ] || { echo "gemm_bench older than common.h: rebuild it"; exit 2; }
  echo "== gemm_bench $(date +%T)"
  timeout -k 10 600 tools/gemm_bench --reps ${REPS:-20} ${SHAPES:+--shapes $SHAPES} ${LIBS} > gpurun_out/${TAG}_gemm.txt 2>&1
  rc=$?; echo "gemm rc=$rc"; cat gpurun_out/${TAG}_gemm.txt | tail -${NTAIL:-60}
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if phase steps || phase core; then
  for a in ${ARCHS:-eres2netv2 eres2net_large ecapa campplus}; do
    timeout -k 10 300 python tools/profile_steps.py --arch $a --json gpurun_out/${TAG}_steps_$a.json > gpurun_out/${TAG}_steps_$a.txt 2>&1
    rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_steps_$a.txt | head -${NSTEP:-1}
    if fatal $rc; then exit $rc; fi
  done
fi
if phase ab; then
  for rep in $(seq ${REPS_AB:-2}); do
    for lib in ${LIBS}; do
      t=$(basename $lib .so)
      for a in ${ARCHS:-eres2netv2}; do
        SPK_HIP_LIB=$lib timeout -k 10 300 python tools/profile_steps.py --arch $a --json gpurun_out/${TAG}_ab_${t}_${a}_$rep.json \
            > gpurun_out/${TAG}_ab_${t}_${a}_$rep.txt 2>&1
        rc=$?; echo "$t rep $rep: $(grep -v amdgpu.ids gpurun_out/${TAG}_ab_${t}_${a}_$rep.txt | head -1)"
        if fatal $rc; then exit $rc; fi
      done
    done
  done
fi
if phase core || phase pmc; then
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== rocprofv3 --pmc $c $(date +%T)"
    timeout -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/${TAG}_pmc_$c -o run --output-format csv -- \
        python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_pmc_$c.log 2>&1
    rc=$?; echo "pmc rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_pmc_$c.log; exit $rc; fi
  done
  python tools/pmc_traffic.py gpurun_out/${TAG}_pmc_FETCH_SIZE gpurun_out/${TAG}_pmc_WRITE_SIZE -o gpurun_out/${TAG}_pmc_traffic.json \
      && cp gpurun_out/${TAG}_pmc_traffic.json profiles/pmc_traffic.json
  echo "== pmc sq $(date +%T)"
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
      -d gpurun_out/${TAG}_pmc_mfma -o run --output-format csv -- python tools/profile_steps.py --arch eres2netv2 > gpurun_out/${TAG}_pmc_mfma.log 2>&1
  rc=$?; echo "pmc sq rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_pmc_mfma.log; exit $rc; fi
  python tools/pmc_mfma.py gpurun_out/${TAG}_pmc_mfma -o gpurun_out/${TAG}_sq_counters.json > gpurun_out/${TAG}_sq_counters.txt 2>&1
  head -12 gpurun_out/${TAG}_sq_counters.txt
fi
if phase core || phase prof; then
  echo "== rocprofv3 stats $(date +%T)"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/${TAG}_prof.log | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if phase core || phase bench; then
  echo "== bench $(date +%T)"
  timeout -k 10 600 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/${TAG}_bench.log | cut -c1-700
fi
if phase workloads; then
  for w in "c1" "c3" "c3 --precision fp16" "models"; do
    t=$(echo $w | tr -c 'a-z0-9\n' '_')
    echo "== workload $w $(date +%T)"
    timeout -k 10 300 python tools/bench_workloads.py $w > gpurun_out/${TAG}_wl_$t.json 2> gpurun_out/${TAG}_wl_$t.err
    rc=$?; head -c 600 gpurun_out/${TAG}_wl_$t.json; echo; if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_wl_$t.err; fi
    if fatal $rc; then exit $rc; fi
  done
  echo "== c4 $(date +%T)"
  timeout -k 10 700 python tools/bench_c4.py > gpurun_out/${TAG}_wl_c4.json 2> gpurun_out/${TAG}_wl_c4.err
  rc=$?; head -c 800 gpurun_out/${TAG}_wl_c4.json; echo; if fatal $rc; then exit $rc; fi
  echo "== c5 $(date +%T)"
  timeout -k 10 500 python tools/bench_diarization.py > gpurun_out/${TAG}_wl_c5.json 2> gpurun_out/${TAG}_wl_c5.err
  rc=$?; head -c 600 gpurun_out/${TAG}_wl_c5.json; echo; if fatal $rc; then exit $rc; fi
fi
echo "== done $(date +%T)"
exit $rc
