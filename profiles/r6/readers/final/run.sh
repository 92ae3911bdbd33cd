# round 6: where one https cluster watch waits — the fixture's senders (sealing, waiting for the
# socket) against the watcher's reader (recv, opening, epoll idle, buffer waits), plain http beside it.
# usage: bash scripts/boxruns/tls_timeline.sh TAG [runs...]   (runs: tls plain tls64 plain64)
set -o pipefail
T=${1:-x}; shift
O=gpurun_out/r6tt_$T
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5"
i=0
for r in "$@"; do
  i=$((i+1))
  case $r in
    tls) X="--api-tls";; plain) X="";;
    tlsboth) X="--api-tls --tls";; tlssink) X="--tls";;
    tlsapart) X="--api-tls --fixture-placement apart";; plainapart) X="--fixture-placement apart";;
    tls64) X="--api-tls --watch-scope discover --namespaces 64";; plain64) X="--watch-scope discover --namespaces 64";;
    r1m32) X="--watch-scope discover --namespaces 64 --set watcher.watch_reader_max_bytes=33554432"; export BENCH_HUB_READERS=1;;
    r2m32) X="--watch-scope discover --namespaces 64 --set watcher.watch_reader_max_bytes=33554432"; export BENCH_HUB_READERS=2;;
    r2m64) X="--watch-scope discover --namespaces 64 --set watcher.watch_reader_max_bytes=67108864"; export BENCH_HUB_READERS=2;;
    r1) X="--watch-scope discover --namespaces 64"; export BENCH_HUB_READERS=1;;
    r2smt) X="--watch-scope discover --namespaces 64"; export BENCH_HUB_READERS=2 BENCH_READERS_SHARE_CORE=1;;
    r1b) X="--watch-scope discover --namespaces 64"; export BENCH_HUB_READERS=1; unset BENCH_READERS_SHARE_CORE;;
    p1) X="--watch-scope discover --namespaces 64 --probe"; export BENCH_HUB_READERS=1; unset BENCH_READERS_SHARE_CORE;;
    p2) X="--watch-scope discover --namespaces 64 --probe"; export BENCH_HUB_READERS=2; unset BENCH_READERS_SHARE_CORE;;
    ns0) X="--watch-scope discover --namespaces 64 --probe"; export BENCH_HUB_READERS=1; unset BENCH_READERS_SHARE_CORE;;
    ns32) X="--watch-scope discover --namespaces 64 --probe --set watcher.watch_reader_max_bytes=33554432"; export BENCH_HUB_READERS=1; unset BENCH_READERS_SHARE_CORE;;
    ns16) X="--watch-scope discover --namespaces 64 --probe --set watcher.watch_reader_max_bytes=16777216"; export BENCH_HUB_READERS=1; unset BENCH_READERS_SHARE_CORE;;
    r2ns16) X="--watch-scope discover --namespaces 64 --probe --set watcher.watch_reader_max_bytes=16777216"; export BENCH_HUB_READERS=2; unset BENCH_READERS_SHARE_CORE;;
    r2ns8) X="--watch-scope discover --namespaces 64 --probe --set watcher.watch_reader_max_bytes=8388608"; export BENCH_HUB_READERS=2; unset BENCH_READERS_SHARE_CORE;;
    d64) X="--watch-scope discover --namespaces 64"; export BENCH_HUB_READERS=1; unset BENCH_READERS_SHARE_CORE;;
    r2m8) X="--watch-scope discover --namespaces 64 --set watcher.watch_reader_max_bytes=8388608"; export BENCH_HUB_READERS=2; unset BENCH_READERS_SHARE_CORE;;
    r2full) X="--watch-scope discover --namespaces 64"; export BENCH_HUB_READERS=2; unset BENCH_READERS_SHARE_CORE;;
    r1m8) X="--watch-scope discover --namespaces 64 --set watcher.watch_reader_max_bytes=8388608"; export BENCH_HUB_READERS=1; unset BENCH_READERS_SHARE_CORE;;
    cl0) X="--probe"; export BENCH_HUB_READERS=1;;
    cl32) X="--probe --set watcher.watch_reader_max_bytes=33554432"; export BENCH_HUB_READERS=1;;
    tls64r1) X="--api-tls --watch-scope discover --namespaces 64"; export BENCH_HUB_READERS=1;;
    tls64r2) X="--api-tls --watch-scope discover --namespaces 64"; export BENCH_HUB_READERS=2;;
    *) echo "unknown run $r"; exit 2;;
  esac
  timeout -k 10 300 $B $X --json-out $O/${i}_$r.json > $O/${i}_$r.out 2> $O/${i}_$r.err || exit $?
done
