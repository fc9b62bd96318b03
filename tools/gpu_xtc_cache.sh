cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_xtc_gpu.py tests/test_gpu_xtc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/xc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/xc_tests.log; [ $rc -ne 0 ] && exit $rc
for C in "" "--xtc-cache"; do
timeout -k 10 300 python -u bench.py --workload c5xtc --align average $C --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/xc_bench$C.json 2> gpurun_out/xc_bench$C.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/xc_bench$C.json'));print('$C', d['value'], d['ms_per_step'], d['stager']['xtc_frames_per_s'])"
done
