#!/bin/bash
# Round 5: same-box A/B of the config-2 step: new defaults (channels-last fp32 encoders, MIOpen
# benchmark mode) with the current find-db and with the pre-batch-12-tuning one, the old defaults.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5/ab
mkdir -p $OUT
export PYTHONUNBUFFERED=1
B="--no-cpu-baseline --no-parity --steps 20 --warmup 5"
pr() { python -c "import json;d=json.load(open('$OUT/$1.json'));print('$1',d['value'],d['ms_per_step'])"; }
timeout -k 10 400 python bench.py $B > $OUT/new.json 2> $OUT/new.err && pr new || exit 1
MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/variants/db_tune2 timeout -k 10 400 python bench.py $B > $OUT/new_db2.json 2> $OUT/new_db2.err && pr new_db2 || exit 1
VFD_CHANNELS_LAST=1 timeout -k 10 400 python bench.py $B --conv-autotune 0 > $OUT/old.json 2> $OUT/old.err && pr old || exit 1
timeout -k 10 400 python bench.py $B --conv-autotune 0 > $OUT/new_imm.json 2> $OUT/new_imm.err && pr new_imm || exit 1
timeout -k 10 400 python bench.py $B > $OUT/new2.json 2> $OUT/new2.err && pr new2 || exit 1
