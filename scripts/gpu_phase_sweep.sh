cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6_wmap && timeout -k 10 900 python scripts/wgrad_inmodel_ab.py --arms wmap=3,wmap=-1 --rounds 8 --steps 4 --warmup 2 > gpurun_out/r6_wmap/inmodel.log 2>&1
