#!/bin/bash
# Round-2 GPU session: GPU test suite, bench (N=1), 2-rank launcher rehearsal (gloo, one GPU),
# rocprofv3 kernel trace. Usage: scripts/gpu_r05.sh TAG [pytest-args...]
TAG=${1:-r05a}
shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())" > $OUT/host.txt
cat /sys/fs/cgroup/cpu.max >> $OUT/host.txt 2>/dev/null
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread "$@" > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -1 $OUT/bench.json | cut -c1-400
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --mode views --steps 5 --warmup 2 --e2e-steps 0 \
    > $OUT/bench_views2_gloo.json 2> $OUT/bench_views2_gloo.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 --train-steps 0 > $OUT/trace.log 2>&1 || exit $?
exit $rc
