cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6_mlpov && timeout -k 10 900 python scripts/wgrad_inmodel_ab.py --arms mlpov=0,mlpov=1 --rounds 6 --steps 4 --warmup 2 > gpurun_out/r6_mlpov/ab.log 2>&1
