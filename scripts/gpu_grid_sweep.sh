# C4 bench under different persistent-grid caps (SPAI_FWD_GRID) and chain counts (SPAI_CHAINS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/grid; mkdir -p $OUT
for cfg in ${CFGS:-"256:2" "192:2" "160:2" "128:2"}; do
  g=${cfg%%:*}; c=${cfg##*:}
  SPAI_FWD_GRID=$g SPAI_CHAINS=$c timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/b_${g}_$c.json 2> $OUT/b_${g}_$c.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/b_${g}_$c.json')); print('grid $g chains $c', round(d['value']/1e6,3), 'M sims/s fwd', round(d['kernel_ms']['evaluate']*1e3,1), 'us leaves', round(d['roofline']['avg_leaves_per_launch']), 'frac', round(d['roofline']['frac'],3), 'chip', round(d['roofline']['chip_frac'],3))"
done 2>&1 | tee $OUT/sweep.txt
