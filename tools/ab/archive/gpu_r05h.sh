# round 5: where the CLI's 3.1 s go (config 2, kmer uniq into /dev/null), finer phases
set -e
mkdir -p gpurun_out
timeout -k 10 300 python tools/clibench.py uniq 3 > gpurun_out/r05h_cli.txt 2>&1 || { tail -20 gpurun_out/r05h_cli.txt; exit 1; }
cat gpurun_out/r05h_cli.txt
