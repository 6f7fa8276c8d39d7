cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_prefetch.py tests/test_gpu_mock.py tests/test_gpu_parity.py -k "prefetch or mock or psrfits" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_pf.log 2>&1; tail -2 gpurun_out/t_pf.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu --e2e-beams 0 --sp-beams 0 --fft-beams 0 --rfi-beams 0 --stream-beams 3 > gpurun_out/b_stream.log 2>&1 || exit 1
tail -1 gpurun_out/b_stream.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stream_beams'])"
HD_QFIX=1 bash scripts/ab_bench.sh 0 || exit 1
