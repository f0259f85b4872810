#!/bin/bash
# Frame batches (pbr_hip_render_frames): the batch tests, then C2 per-frame vs batch, then the C2 shard
# projection with and without batches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/batch_tests.log 2>&1
rc=$?; tail -4 gpurun_out/batch_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in ${CONFIGS:-C2}; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 5 --no-cpu-baseline --no-model --per-frame > gpurun_out/bench_perframe_$cfg.log 2>&1 || exit 4
  timeout -k 10 300 python -u bench.py --config $cfg --steps 5 --no-cpu-baseline --no-model > gpurun_out/bench_batch_$cfg.log 2>&1 || exit 4
  for m in perframe batch; do tail -1 gpurun_out/bench_${m}_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $m', d['ms_per_step'], 'ms', d['value'], 'Msamples/s; serial', d['roofline']['serial_frame_ms'])"; done
done
if [ -n "${SHARDS:-}" ]; then
  timeout -k 10 300 python -u tools/shard_projection.py --config C2 --batch 0 --json gpurun_out/shard_c2_perframe.json > gpurun_out/shard_c2_perframe.log 2>&1 || exit 5
  timeout -k 10 300 python -u tools/shard_projection.py --config C2 --batch 5 --json gpurun_out/shard_c2_batch.json > gpurun_out/shard_c2_batch.log 2>&1 || exit 5
  tail -4 gpurun_out/shard_c2_perframe.log gpurun_out/shard_c2_batch.log
fi
