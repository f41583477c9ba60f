cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pk3
EELG_LIB=$R/variants/libeelg_pk3.so timeout -k 10 300 python3 -m pytest $R/tests/test_gpu_parity.py -q -x -k "product or symcon or model_forward" --timeout 200 --timeout-method thread > $R/gpurun_out/pk3/tests.log 2>&1 &&
timeout -k 10 200 python3 $R/tools/kbench.py --reps 20 --only "sc_" > $R/gpurun_out/pk3/k_main.txt 2>&1 &&
EELG_LIB=$R/variants/libeelg_pk3.so timeout -k 10 200 python3 $R/tools/kbench.py --reps 20 --only "sc_" > $R/gpurun_out/pk3/k_pk3.txt 2>&1
