#!/bin/bash
# r4a (tests + moments / decblk benches) then r4b (PMC passes: p16, f32shift), one box.
set -u
cd "$(dirname "$0")/.."
bash scripts/gpu_r4a.sh r4a && bash scripts/gpu_r4b.sh r4b
