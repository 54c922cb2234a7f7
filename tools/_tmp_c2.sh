set -o pipefail
O=gpurun_out/r05c2; mkdir -p $O
for i in 1 2 3; do
  for ah in 0 1; do
    timeout -k 10 200 python tools/ab_variants.py --scene scenes/cornell_box.scene.json --width 512 --height 512 --spp 64 --variants 0 --block 8 --rounds 2 --ahead $ah > $O/c2_a${ah}_$i.log 2>&1 || { echo FATAL; exit 5; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); v=d['variants']['0']; print(sys.argv[2], v['ran'], v['median_ms'], min(v['ms']))" $O/c2_a${ah}_$i.log a$ah
  done
done
