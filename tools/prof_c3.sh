GPEMU_CONCURRENT_TRIES=1 timeout -k 10 300 python3 -m cProfile -s cumtime tools/train_c3.py --tries 1 > gpurun_out/c3_prof.txt 2>&1
