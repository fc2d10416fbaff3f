cd $GRAFT_REPO_ROOT
for path in auto generic windowed; do RHMC_KERNEL=$path timeout -k 10 300 python3 bench.py --workload C3 --chains 2048 --leap 50 --steps 3 --warmup 1 --no-cpu > gpurun_out/c3_$path.log 2>&1 || exit $?; done
