# K1 ablations at 8192x8192: every gpurun_var/* build (tools/variant.sh) timed with tools/kab.sh
set -o pipefail
V="$(ls -d gpurun_var/*/ | sed 's#/$##')"
KB_SIZE=8192x8192 bash tools/kab.sh abl $V && grep -E "fdct|libmyyuv" gpurun_out/kab_abl.txt
