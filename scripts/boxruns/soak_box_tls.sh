# round 6: saturated https soak on the box, final tree — 14 minutes of 10-step chunks over the
# TLS 1.3 record layer (fixture: sealed records sent with sendfile), each chunk checked exactly-once
set -o pipefail
O=gpurun_out/${1:-r6soak_tls}
mkdir -p $O
timeout -k 10 1080 python3 bench.py --api-tls --soak-minutes 14 --json-out $O/soak14_tls.json > $O/soak14_tls.out 2> $O/soak14_tls.err
