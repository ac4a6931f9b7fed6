cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6_dkdv && timeout -k 10 900 python scripts/wgrad_inmodel_ab.py --arms dkpk=1,dkpk=0 --rounds 8 --steps 4 --warmup 2 > gpurun_out/r6_dkdv/inmodel.log 2>&1
