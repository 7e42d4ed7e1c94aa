# Round 5: repeated multi-session renders of config 2 on one GPU (tools/ngpu_parity.py) under
# PT_TUNE variants, with the lost-chain diagnostics (shortlog=1) on stderr.  Output: gpurun_out/np
mkdir -p gpurun_out/np
timeout -k 10 500 python3 tools/ngpu_parity.py --cfg c2 --ngpu ${NGPU:-4} --repeat ${REPEAT:-12} --tunes ${TUNES:-same_device=1,early_wg=8,shortlog=1} > gpurun_out/np/np.jsonl 2> gpurun_out/np/np.err; echo rc=$?
python3 - <<'PY'
import json, collections
c = collections.Counter()
for l in open("gpurun_out/np/np.jsonl"):
    d = json.loads(l); c[(d["tune"], d["ok"])] += 1
for k, v in sorted(c.items()): print(k, v)
PY
grep -h "short: done" gpurun_out/np/np.err | head -20
