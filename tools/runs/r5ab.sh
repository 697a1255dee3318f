# round 5 diagnostic: the fused decoder's VALU split, from SQ counters of
# ablation builds (transform skipped: build_var/ablxf; symbol loop skipped:
# build_var/ablsym; wrong output by design, never shipped) against HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in base ablxf ablsym; do
  timeout -k 10 600 bash tools/sq_counters.sh r5ab_$v build_var/$v > /dev/null 2>&1 || { echo SQ_FAILED $v; exit 1; }
  echo "== $v"; python3 tools/sq_report.py r5ab_$v 2>/dev/null | awk '/^== decode_idct/{f=1} /^== /&&!/decode_idct/{f=0} f' | grep -E "SQ_INSTS_VALU|SQ_WAVES|SQ_INSTS_LDS|SQ_WAVE_CYCLES|VALU/wave"
done
