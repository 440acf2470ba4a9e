# Round 6 session a: baseline forward numbers on one box -- phase stamps (diag
# build), per-k-step stamps of a steady-state S = 8 conv (k-step diag build), and
# the isolated forward at the streamed schedule's leaf counts (one and two chains)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r06a} && mkdir -p $O
SPAI_LIB=build_exp/libspai_diag.so timeout -k 10 300 python3 scripts/net_phases.py > $O/phases.txt 2>&1 || { tail -20 $O/phases.txt; exit 1; }
cat $O/phases.txt
SPAI_LIB=build_exp/libspai_kstep.so timeout -k 10 300 python3 scripts/net_kstep.py 8 5 4 > $O/kstep.txt 2>&1 || { tail -20 $O/kstep.txt; exit 1; }
cat $O/kstep.txt
timeout -k 10 300 python3 scripts/fwd_sweep.py --counts 1024,1539,2048,3078,4096 --conc 2 > $O/sweep_conc2.txt 2>&1 || { cat $O/sweep_conc2.txt; exit 1; }
cat $O/sweep_conc2.txt
