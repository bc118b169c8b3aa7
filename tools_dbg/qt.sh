#!/bin/bash
# one parity test under several kernel configurations: qt.sh "<pytest -k expr>" "name:ENV=V,ENV=V" ...
cd $GRAFT_REPO_ROOT
k="$1"; shift
for spec in "$@"; do
  IFS=':' read -r name envs <<< "$spec"
  echo "== $name"; env ${envs//,/ } timeout -k 10 120 python -m pytest tests/test_gpu_parity.py -m gpu -q -k "$k" 2>&1 | grep -E "passed|failed|L-inf" | tail -3
done
