# the product int8 kernel with and without the IgemmZ moduli-batch prologue (microbench A/B on
# one box; igemm_FULL_PREZB is built from the sources before the IgemmZ commit)
set -o pipefail
R=gpurun_out/r04_prezb
mkdir -p $R
cd "$GRAFT_REPO_ROOT/tools/microbench"
for i in 1 2 3; do
  for v in FULL FULL_PREZB EPI_LDS; do
    timeout -k 10 120 ./igemm_$v >> ../../$R/prezb.txt 2>&1 || exit 1
  done
done
