# Clean-checkout check: the committed tree alone (git archive HEAD, no built
# or untracked files) builds with build() and passes smoke() on the MI355X box.
set -o pipefail
mkdir -p gpurun_out
D=$(mktemp -d /tmp/cleanco.XXXXXX)
tar xf clean_checkout.tar -C $D
cd $D
ls template-matching-and-regression-mapreduce_amd/*.so template-matching-and-regression-mapreduce_amd/exp_ref.bin 2>/dev/null && { echo "built files present in the archive"; exit 1; }
timeout -k 10 900 python -c "import __graft_entry__ as g; g.build()" > $GRAFT_REPO_ROOT/gpurun_out/clean_build.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/clean_build.log; exit 1; }
tail -3 $GRAFT_REPO_ROOT/gpurun_out/clean_build.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $GRAFT_REPO_ROOT/gpurun_out/clean_smoke.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/clean_smoke.log; exit 1; }
tail -3 $GRAFT_REPO_ROOT/gpurun_out/clean_smoke.log
