cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/sweep_env.sh r05e C3 "GPC_CBAND_MERGE=4 GPC_CBAND_MERGE=1 GPC_CBAND_MERGE=2 GPC_CBAND_MERGE=3" --steps 20 || exit 1
bash tools/sweep_env.sh r05e C4 "GPC_CBAND_MERGE=4 GPC_CBAND_MERGE=1 GPC_CBAND_MERGE=2" --steps 20 || exit 1
bash tools/sweep_env.sh r05e C2 "GPC_CBAND_MERGE=4 GPC_CBAND_MERGE=1" --steps 20 || exit 1
