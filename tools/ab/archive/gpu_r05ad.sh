# round 5: `kmer uniq` / `count` on config 2's 1 GB FASTA into /dev/null after device batches stopped allocating a
# size-long record list each (1000 batches of 1 M k-mers)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05ad_tests.log 2>&1 || { tail -40 gpurun_out/r05ad_tests.log; exit 1; }
tail -1 gpurun_out/r05ad_tests.log
timeout -k 10 400 python tools/clibench.py uniq 3 > gpurun_out/r05ad_uniq.txt 2>&1 || { tail -20 gpurun_out/r05ad_uniq.txt; exit 1; }
tail -3 gpurun_out/r05ad_uniq.txt
timeout -k 10 400 python tools/clibench.py count 2 > gpurun_out/r05ad_count.txt 2>&1 || { tail -20 gpurun_out/r05ad_count.txt; exit 1; }
tail -2 gpurun_out/r05ad_count.txt
