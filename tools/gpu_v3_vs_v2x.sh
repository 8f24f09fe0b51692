cd $GRAFT_REPO_ROOT
OUT=gpurun_out/v3_vs_v2x.jsonl; mkdir -p gpurun_out; : > $OUT
for c in ds2_mixed mixed w8a8 w4a4; do for gg in gate_up down; do
  timeout -k 10 200 python tools/kbench.py --cfg $c --gg $gg --variants 8,5 --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/v3ab.err || exit 1
done; done
cut -c1-130 $OUT
