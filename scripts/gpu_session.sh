#!/bin/bash
# The one GPU session script (run on the box from the repo root, through gpurun).  Steps, in the order given:
#   T=<tag> STEPS="tests bench ab prof profsugar pairs sq sugar" [LIBS="name=path ..."] [AB_ARGS="<bench.py args>"] \
#     [AB_ROUNDS=2] [TESTS="tests/..."] [TEST_TIMEOUT=300] bash scripts/gpu_session.sh
#   tests  pytest -m gpu (one process, per-test time limit)      -> gpurun_out/<T>_tests.log
#   bench  bench.py with the driver's defaults                    -> gpurun_out/<T>_bench.json
#   sugar  bench.py --workload sugar (C5)                          -> gpurun_out/<T>_sugar.json
#   ab     the LIBS builds alternated AB_ROUNDS times (GSR_HIP_LIB) -> gpurun_out/<T>_ab_<name>_<round>.json
#   prof   rocprofv3 kernel trace + FETCH / WRITE / VALU passes   -> gpurun_out/prof_<T>/ (profiles/summarize.py)
#   profsugar  the same for bench.py --workload sugar              -> gpurun_out/prof_<T>_sugar/
#   pairs  device-counted blend pairs (diagnostic build)          -> gpurun_out/pairs_<T>[_sugar].json
#   sq     SQ counter passes of the blends                         -> gpurun_out/sq_<T>/ (profiles/sq_summary.py)
# Every GPU step runs under its own time limit; the first failing step ends the session.
set -o pipefail
mkdir -p gpurun_out
T=${T:-s}
AB_ARGS=${AB_ARGS:-"--steps 10 --warmup 3 --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"}
for step in ${STEPS:-tests bench}; do
  case $step in
    tests)
      timeout -k 10 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -rf --timeout ${TEST_TIMEOUT:-300} --timeout-method thread \
        > gpurun_out/${T}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
      tail -3 gpurun_out/${T}_tests.log ;;
    bench)
      timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 1
      python scripts/bench_summary.py gpurun_out/${T}_bench.json ;;
    sugar)
      timeout -k 10 400 python -u bench.py --workload sugar --no-cpu-baseline --no-knn --extra-lines none \
        > gpurun_out/${T}_sugar.json 2> gpurun_out/${T}_sugar.log || exit 1
      python scripts/bench_summary.py gpurun_out/${T}_sugar.json ;;
    ab)
      for round in $(seq 1 ${AB_ROUNDS:-2}); do
        for spec in $LIBS; do
          name=${spec%%=*}; lib=${spec#*=}
          GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $AB_ARGS > gpurun_out/${T}_ab_${name}_${round}.json \
            2> gpurun_out/${T}_ab_${name}_${round}.log || exit 1
          python scripts/bench_summary.py gpurun_out/${T}_ab_${name}_${round}.json
        done
      done ;;
    prof)
      bash profiles/run_profiles.sh $T || exit 1
      python profiles/summarize.py $T > gpurun_out/${T}_summarize.log 2>&1 || exit 1 ;;
    profsugar)
      bash profiles/run_profiles.sh ${T}_sugar --workload sugar || exit 1
      python profiles/summarize.py ${T}_sugar > gpurun_out/${T}_sugar_summarize.log 2>&1 || exit 1 ;;
    pairs)  # device-counted pairs (diagnostic build: make -C threestudio-3dgs_amd/csrc diag, CPU side)
      timeout -k 10 300 python -u profiles/diag_pairs.py $T > gpurun_out/${T}_pairs.log 2>&1 || exit 1
      timeout -k 10 300 python -u profiles/diag_pairs.py $T sugar > gpurun_out/${T}_pairs_sugar.log 2>&1 || exit 1 ;;
    sq)
      bash profiles/run_sq.sh $T || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session $T done"
