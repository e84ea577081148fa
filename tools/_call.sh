set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
# same library (stride-aware), records laid out as three arrays (soa) or one interleaved array (aos)
for c in str_card1e8 str_card1e5; do for rep in 1 2; do for v in soa aos; do
  echo "== $v $c rep $rep" >> gpurun_out/r04x_ab.log
  SDP_AB_SOA_RECORDS=$([ $v = soa ] && echo 1 || echo 0) timeout -k 10 240 python -u tools/kbench.py group 1000000000 2 $c 2>&1 \
      | grep -v amdgpu.ids | tail -n +3 >> gpurun_out/r04x_ab.log || exit 1
done; done; done
grep -E "==|bytes" gpurun_out/r04x_ab.log
