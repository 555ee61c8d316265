export TFIDF_DEBUG=1
B="python -u bench.py --no-queries --no-e2e --cpu-sample 0 --prose 1"
for sw in "3 1" "10 2" "10 1" "3 2"; do set -- $sw
timeout -k 10 300 $B --steps $1 --warmup $2 > gpurun_out/pb.json 2>gpurun_out/pb.err || exit 1
python3 -c "import json; r=json.loads(open('gpurun_out/pb.json').read().strip().splitlines()[-1]); print('steps $1 warmup $2 tokenize %.3f step %.3f rebuilds %s' % (r['phases_ms']['ms_tokenize'], r['ms_per_step'], r.get('hash_rebuilds')))"
done
