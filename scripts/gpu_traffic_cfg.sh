#!/bin/bash
# Per-op HBM traffic (FETCH_SIZE and WRITE_SIZE passes, separate runs) of the step at the configs
# given: `scripts/gpu_traffic_cfg.sh 2 3 5` -> gpurun_out/traffic_c<N>/ and traffic_config<N>.json
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for C in "$@"; do
  OUT=$R/gpurun_out/traffic_c$C
  mkdir -p $OUT
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python $R/bench.py --config $C --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $OUT/fetch.log 2>&1) || exit $?
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python $R/bench.py --config $C --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $OUT/write.log 2>&1) || exit $?
  python tools/traffic_from_pmc.py $(ls $OUT/fetch/*/*counter_collection.csv $OUT/fetch/*counter_collection.csv 2>/dev/null | head -1) \
    $(ls $OUT/write/*/*counter_collection.csv $OUT/write/*counter_collection.csv 2>/dev/null | head -1) > gpurun_out/traffic_config$C.json || exit $?
  echo "config $C traffic ok"
  rm -rf $OUT/fetch $OUT/write
done
