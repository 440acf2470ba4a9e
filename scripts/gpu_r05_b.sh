# Round 5 session b: numerics and forward-alone timing of the split-K 8-wave
# forward (SPAI_W8) against the default build, at group sizes forced to S = 4
# (SPAI_ONLY_S=4 in both) and over S <= 5 (all-S W8 build vs default).
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05b} && mkdir -p $O
D=self-play-ai_amd/libspai.so
timeout -k 10 300 python3 scripts/variant_check.py $D,build_exp/libspai_s4.so,build_exp/libspai_w8s4.so --counts 1000,900 > $O/check_s4.txt 2>&1; rc=$?; cat $O/check_s4.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/variant_check.py $D,build_exp/libspai_w8.so --counts 512,768,1000,1280,60 > $O/check_w8.txt 2>&1; rc=$?; cat $O/check_w8.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 scripts/fwd_sweep.py --libs build_exp/libspai_s4.so,build_exp/libspai_w8s4.so --counts 900,1000 > $O/sweep_s4_$r.txt 2>&1 || { cat $O/sweep_s4_$r.txt; exit 1; }
  cat $O/sweep_s4_$r.txt
  timeout -k 10 300 python3 scripts/fwd_sweep.py --libs $D,build_exp/libspai_w8.so --counts 60,512,768,1000,1280 > $O/sweep_all_$r.txt 2>&1 || { cat $O/sweep_all_$r.txt; exit 1; }
  cat $O/sweep_all_$r.txt
done
