cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/m5; mkdir -p $O
timeout -k 10 400 python3 -m cProfile -o $O/sfd.prof bench.py --config c5 --integrator sfd --spp 256 --steps 1 --warmup 1 --cpu-budget 0 > $O/sfd.json 2> $O/sfd.log || { tail $O/sfd.log; exit 1; }
python3 -c "
import pstats; p=pstats.Stats('$O/sfd.prof'); p.sort_stats('cumulative').print_stats(35)" > $O/prof.txt
head -80 $O/prof.txt | tail -60
