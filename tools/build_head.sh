#!/bin/bash
# Build the committed HEAD's library into orion-kmer_amd/build_head (A/B baseline).
set -e
cd "$(dirname "$0")/.."
rm -rf /tmp/okm_head_wt
git worktree add -f /tmp/okm_head_wt HEAD -q
make -s -j8 -C /tmp/okm_head_wt/orion-kmer_amd > /dev/null
mkdir -p orion-kmer_amd/build_head
cp /tmp/okm_head_wt/orion-kmer_amd/build/liborion_kmer.so orion-kmer_amd/build_head/
git worktree remove --force /tmp/okm_head_wt
