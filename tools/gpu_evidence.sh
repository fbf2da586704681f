# Round evidence: tools/gpu4.sh (tests, smoke, PMC c2/c3, rocprof kernel stats c2/c3) then tools/gpu5.sh (bench lines).
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu4.sh && bash tools/gpu5.sh
