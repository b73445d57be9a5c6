cd $GRAFT_REPO_ROOT
bash tools/gpu_session.sh r05g tests smoke bench kt
