cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/morton
timeout -k 10 200 python3 $R/tools/kbench.py --reps 20 --only "tp_|segment_sum gxe" > $R/gpurun_out/morton/base.txt 2>&1 &&
timeout -k 10 200 python3 $R/tools/kbench.py --reps 20 --only "tp_|segment_sum gxe" --morton > $R/gpurun_out/morton/morton.txt 2>&1
