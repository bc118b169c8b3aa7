#!/bin/bash
# Re-tune of the secondary kernel's schedule constants at round-6 HEAD (PRIM/NODE steps per iteration, refill
# threshold, PRIM bias): C4 bench per build, twice.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="${T:-cur p3 p5 n5 n8 r16 r32 b60 b85}"
bash tools/ab_run.sh $T && python3 tools/ab_summary.py $T && bash tools/ab_run.sh $T && python3 tools/ab_summary.py $T
