# Round-6 final build, part 1: the -m gpu suite (stop on failure), then C2 and C3 measured (tools/r6_measure.sh)
set -o pipefail
OUT=gpurun_out/r6_gpu_tests.log TMO=900 bash tools/r6_tests.sh || exit 1
CONFIGS="C2 C3" bash tools/r6_measure.sh
