set -o pipefail
bash tools/gpu_encfile.sh r04n 8 && bash tools/gpu_encfile_prof.sh r04n_prof && BPE355_TRACE=1 timeout -k 10 300 python tools/enc_bench.py > gpurun_out/r04n/enc_bench.log 2>&1; tail -2 gpurun_out/r04n/enc_bench.log
