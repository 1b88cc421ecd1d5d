cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for sc in demo random:1; do
  timeout -k 10 400 python -u scripts/sched_probe.py --scene $sc --rounds 4 --xcd-chunks c,0,16,17,18,19,20 0:c:c 1:c:c 2:c:c 3:c:c 4:c:c 5:c:c > gpurun_out/latin_$sc.jsonl 2> gpurun_out/latin_err.log || { tail gpurun_out/latin_err.log; exit 1; }
  echo "== $sc"; python3 -c "
import json,sys
for l in open('gpurun_out/latin_$sc.jsonl'):
    d=json.loads(l); c=d['committed'][1]
    print('L%d'%d['level'], 'committed lc', (c>>26)&31, [(t, (o>>26)&31) for t,v,o in d['ms_variant_order']])"
done
