#!/bin/bash
# round-2 profile: kernel trace + separate FETCH_SIZE / WRITE_SIZE passes
set -e
cd $GRAFT_REPO_ROOT
bash scripts/profile_round.sh r2u "--steps 20 --warmup 5 --no-cpu-baseline --retrieval-steps 5 --sweep , --c3-steps 2 --e2e-steps 3"
