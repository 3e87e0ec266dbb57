set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r3_knn2.sh || exit $?
bash tools/gpu/r3_engine_prof.sh || exit $?
