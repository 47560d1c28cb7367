#!/usr/bin/env bash
# Second A/B of the split template build: alternating headline-shard runs.
set -u
bash tools/ab.sh c4of8 libtfrg_split.so libtfrg.so libtfrg_split.so libtfrg.so libtfrg_split.so libtfrg.so libtfrg_split.so libtfrg.so || exit 1
