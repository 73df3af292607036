set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 600 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_walk.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6b/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r6b/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ab_opts.py C2 10000000 pipe_segs=1 - pipe_segs=2 pipe_segs=8 pipe_segs=4,write_bpc=1 pipe_segs=8,write_bpc=1 > gpurun_out/r6b/ab.txt 2>&1; rc=$?; cat gpurun_out/r6b/ab.txt; exit $rc
