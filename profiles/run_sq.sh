#!/bin/bash
# SQ (wave / issue / LDS) counters of the hot kernels, one rocprofv3 --pmc pass per counter group
# (counter collection kept apart from tracing).  Run on the GPU box from the repo root:
#   bash profiles/run_sq.sh <tag>   -> gpurun_out/sq_<tag>/g*/...counter_collection.csv
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/sq_${1:-r01}
ARGS=${SQ_ARGS:-"--steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-knn --per-view-views 0 --extra-lines none"}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/g$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT.g$i.log 2>&1
done
echo done
