# round 5: zero-copy writer default + chunked file loader: output-byte tests, the CLI on config 2
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_devformat.py tests/test_gpu_parity.py tests/test_host_api.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05j_tests.log 2>&1 || { tail -40 gpurun_out/r05j_tests.log; exit 1; }
tail -1 gpurun_out/r05j_tests.log
timeout -k 10 300 python tools/clibench.py uniq 2 > gpurun_out/r05j_cli.txt 2>&1 || { tail -20 gpurun_out/r05j_cli.txt; exit 1; }
timeout -k 10 300 python tools/clibench.py count 2 >> gpurun_out/r05j_cli.txt 2>&1 || { tail -20 gpurun_out/r05j_cli.txt; exit 1; }
cat gpurun_out/r05j_cli.txt
