#!/usr/bin/env bash
# r5: the randomised parity soaks on the final build (exact records bitwise vs the oracle,
# harmonic ties explained; windows / Float32 storage / device shards / faint states).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5ak
mkdir -p $O
timeout -k 10 330 python -u tools/soak_exact.py --seconds 270 --seed 2031 > $O/soak_exact.jsonl 2> $O/soak_exact.err || { tail -5 $O/soak_exact.jsonl; tail -20 $O/soak_exact.err; exit 1; }
tail -1 $O/soak_exact.jsonl
timeout -k 10 330 python -u tools/soak_more.py --seconds 270 --seed 31 > $O/soak_more.jsonl 2> $O/soak_more.err || { tail -5 $O/soak_more.jsonl; tail -20 $O/soak_more.err; exit 1; }
tail -1 $O/soak_more.jsonl
