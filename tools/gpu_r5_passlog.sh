# Round 5: per-round logs of one rank's 256-spp pass (tools/pass_log.py) at ranks of WORLDS
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r5p || exit 1
O=gpurun_out/r5p
for w in ${WORLDS:-1 4 8}; do
  for r in ${RANKS:-0}; do
    [ $r -ge $w ] && continue
    timeout -k 10 300 python3 tools/pass_log.py --world $w --rank $r --level ${LEVEL:-3} ${PTUNE:+--tune "$PTUNE"} > $O/${TAG:-p}_w${w}_r${r}.txt 2> $O/${TAG:-p}_w${w}_r${r}.err || { echo FAIL w$w r$r; tail -20 $O/${TAG:-p}_w${w}_r${r}.err; exit 1; }
    tail -1 $O/${TAG:-p}_w${w}_r${r}.txt
  done
done
