set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for L in xso/bin.so pysicalbasedraytracer_amd/libpbr_hip.so xso/q6.so xso/q5.so; do
  timeout -k 10 120 python -u tools/tune_wavefront.py --config C2 --steps 5 --lib $L --ref-file gpurun_out/c2ref.npy || exit 1
done
for L in xso/bin.so pysicalbasedraytracer_amd/libpbr_hip.so; do
  timeout -k 10 200 python -u tools/tune_wavefront.py --config C3 --steps 2 --lib $L --ref-file gpurun_out/c3ref.npy || exit 1
done
