# saturated soak on the box, plain http, current tree — 16 minutes of 10-step chunks, each checked exactly-once
set -o pipefail
O=gpurun_out/${1:-r6soak}
mkdir -p $O
timeout -k 10 1120 python3 bench.py --soak-minutes 16 --json-out $O/soak16.json > $O/soak16.out 2> $O/soak16.err
