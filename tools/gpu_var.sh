set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in base sleep20 nopoll nowpe; do
  lib=wrinklefree-inference-engine_amd/lib/libwfbitnet_stamps_$n.so
  [ $n = base ] && lib=wrinklefree-inference-engine_amd/lib/libwfbitnet_stamps.so
  WF_STAMPS_LIB=$lib timeout -k 10 200 python -u tools/stamps_graph.py --ctx 1024 --reps 20 > gpurun_out/stamps_$n.txt 2>&1 || exit 1
  echo "== $n"; grep "^attn\|step_ms" gpurun_out/stamps_$n.txt | cut -c1-300
done
bash tools/prof_prefill.sh r05a
