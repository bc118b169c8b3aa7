cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/m1; mkdir -p $O
timeout -k 10 300 python3 bench.py --cpu-budget 0 --flops 0 --steps 3 > $O/b_1e6.json 2> $O/b_1e6.log || exit 1
timeout -k 10 300 python3 bench.py --cpu-budget 0 --flops 0 --steps 3 --t-eps 0 > $O/b_0.json 2> $O/b_0.log || exit 1
echo ok
