cd $GRAFT_REPO_ROOT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
mkdir -p gpurun_out; OUT=gpurun_out/trace_epi.jsonl; : > $OUT
for d in 2048,2048,8192 4096,4096,8192 8192,8192,8192 8192,8192,2048; do
  for cfg in w8a8 fp16; do
    timeout -k 10 120 python tools/tile_trace.py --cfg $cfg --dense $d --variant-name abl_v2x_edma_trace >> $OUT 2>>gpurun_out/trace_epi.err || exit 1
  done
done
