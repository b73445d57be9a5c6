cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/sweep_env.sh r05f C3 "GPC_CBAND_MERGE=0 GPC_CBAND_MERGE=1 X=adaptive" --steps 20 || exit 1
bash tools/sweep_env.sh r05f C4 "GPC_CBAND_MERGE=0" --steps 20 || exit 1
bash tools/sweep_env.sh r05f C2 "GPC_CBAND_MERGE=3 GPC_CBAND_MERGE=4" --steps 20 || exit 1
bash tools/sweep_env.sh r05f C1 "GPC_CBAND_MERGE=0 GPC_CBAND_MERGE=3 GPC_CBAND_MERGE=4" --steps 20 || exit 1
