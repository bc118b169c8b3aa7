#!/bin/bash
# Round-6 A/B: the chord band (8 / 5 eps c / off) on the C4 bench line, and the light rays' share of the secondary
# node steps (VR_DIAG_LIGHT build's counters).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
bash tools/ab_run.sh cur nob b5
python3 tools/ab_summary.py cur nob b5
bash tools/ab_run.sh cur nob b5
python3 tools/ab_summary.py cur nob b5
VR_LIB_PATH=$PWD/_ab/dlight/libvr_hip.so timeout -k 10 300 python3 tools/diag_c4.py --frames 1 --counts 1 > gpurun_out/ab/dlight.json 2> gpurun_out/ab/dlight.log
timeout -k 10 300 python3 tools/diag_c4.py --frames 1 --counts 1 > gpurun_out/ab/dcur.json 2> gpurun_out/ab/dcur.log
python3 -c "
import json
for t in ('dlight','dcur'):
    d=json.load(open(f'gpurun_out/ab/{t}.json')); print(t, d['slow_rays'], d['work']['secondary'])"
