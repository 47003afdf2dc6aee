set -o pipefail
O=gpurun_out/r3_g2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_seams.py tests/test_gpu_sharded.py tests/test_gpu_pipeline.py tests/test_gpu_batch.py -x -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config5 --no-spectral --no-resample --no-upload > $O/b1.json 2> $O/b1.err || { echo "bench1 failed"; tail -20 $O/b1.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b1.json'));print('N1', d['value'], d['ms_per_step'])"
NC_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-config5 --no-spectral --no-resample --no-upload --no-ibi > $O/b2.json 2> $O/b2.err || { echo "bench2 failed"; tail -30 $O/b2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b2.json'));print('N2', d['value'], d['ms_per_step'], d['modes'])"
NC_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --steps 5 --warmup 2 --no-cpu-baseline --no-config5 --no-spectral --no-resample --no-upload --no-ibi > $O/b4.json 2> $O/b4.err || { echo "bench4 failed"; tail -30 $O/b4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b4.json'));print('N4', d['value'], d['ms_per_step'], d['modes'])"
