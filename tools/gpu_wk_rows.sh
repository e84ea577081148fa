cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in 125000000 1000000000; do for w in 1 2 3; do
timeout -k 10 300 python -u bench.py --rows $r --steps 3 --warmup 1 --no-cpu-baseline --workers $w > gpurun_out/wk_${r}_$w.json 2> gpurun_out/wk_${r}_$w.err || { tail -5 gpurun_out/wk_${r}_$w.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/wk_${r}_$w.json'));print($r,$w,d['ms_per_step'])"
done; done
