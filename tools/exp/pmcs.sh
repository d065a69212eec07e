cd $GRAFT_REPO_ROOT
bash tools/exp/pmc.sh cam_def default C3 --no-lights --bounces 0 &&
bash tools/exp/pmc.sh cam_o2 o2 C3 --no-lights --bounces 0 &&
bash tools/exp/pmc.sh full_def default C3 &&
bash tools/exp/pmc.sh full_o1 o1 C3
