#!/usr/bin/env bash
# Interleaved A/B of bench variants on one box: round 2's bench + library (ab/r2, commit f8607b6), round 3's closing
# HEAD (ab/head), and the working tree (cur), each optionally with env knobs (cur:K=V,K2=V2).
# usage: scripts/ab_variants.sh CONFIG ROUNDS "head cur cur:NH_TAIL_RR_WAVES=1" [extra bench args]
# prints per run: Msamples/s, every roofline stage's ms / launches / rate, and the tail profile when present
set -u
cfg=$1; n=$2; variants=$3; shift 3
mkdir -p gpurun_out
for i in $(seq 1 $n); do
  for v in $variants; do
    name=${v%%:*}; knob=""; [ "$v" != "$name" ] && knob=$(echo "${v#*:}" | tr ',' ' ')
    b=bench.py; [ $name != cur ] && b=ab/$name/bench.py
    tag=$(echo "${cfg}_$v" | tr ':=,/.' '_____')
    extra=""; [ $name = cur ] && extra="--strong-spp 0 --no-extras"
    env $knob timeout -k 10 300 python $b --config $cfg --steps 4 --warmup 1 --no-cpu --no-denoise --traversal-1m-steps 0 \
      $extra "$@" > gpurun_out/ab_$tag$i.log 2>&1 || { echo "fail $v$i"; tail -5 gpurun_out/ab_$tag$i.log; exit 99; }
    python3 - "$cfg $v$i" "gpurun_out/ab_$tag$i.log" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][0])
r = d.get("roofline") or {}
st = r.get("stages", {})
parts = [f"{k} {v['ms']}ms/{v['launches']} {round(v['global_gbs'] / 8000, 4)}" for k, v in st.items()]
tb = sum(v["global_bytes_per_launch"] * v["launches"] for k, v in st.items() if k in ("trace", "extend", "shadow"))
tms = sum(v["ms"] for k, v in st.items() if k in ("trace", "extend", "shadow"))
tp = r.get("tail_profile")
print(sys.argv[1], "Msamples/s", d["value"], "ms/step", d["ms_per_step"], "| splat", r.get("splat_ms_per_launch"), "ms/chunk |", "; ".join(parts),
      f"| traversal (both queries) frac {tb / (tms * 1e-3) / 8e12:.4f}" if tms else "",
      f"| tail chain {tp['longest_chain_bounces']} cyc/bounce {tp['cycles_per_bounce']}" if tp else "",
      f"| coop bounces {tp['coop_bounces']} cyc/bounce {tp['coop_cycles_per_bounce']}" if tp and "coop_bounces" in tp else "")
PY
  done
done
