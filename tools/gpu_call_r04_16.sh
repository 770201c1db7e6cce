cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
PROF_WHICH=mnist TAG=r04_h ISSUE=1 ONLY_ISSUE=1 bash tools/pmc_kernels.sh
python tools/pmc_summary.py $O/pmc_r04_h_v $O/pmc_r04_h_m $O/pmc_r04_h_w --json $O/r04_h_pmc_issue_raw.json > $O/r04_h_pmc_issue_raw.txt || exit 3
python tools/pmc_issue.py $O/r04_h_pmc_issue_raw.json --out $O/r04_h_pmc_issue.json > $O/r04_h_pmc_issue.txt || exit 3
cat $O/r04_h_pmc_issue.txt
rm -rf $O/pmc_r04_h_*/
