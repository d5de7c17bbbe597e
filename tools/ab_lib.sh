#!/bin/bash
# A/B of two in-tree builds on ONE box: alternates tools/tune_route.py runs between the default
# library and $2 (WQ_LIBRARY), so box-to-box variance does not enter the comparison.
# Usage: bash tools/ab_lib.sh <tag> <other .so> [tune_route args...]
set -uo pipefail
T=$1; B=$2; shift 2
O=gpurun_out
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u tools/tune_route.py "$@" > $O/${T}_A$i.json 2>&1 || { tail $O/${T}_A$i.json; exit 1; }
  echo "A$i $(tail -1 $O/${T}_A$i.json)"
  WQ_LIBRARY=$B timeout -k 10 300 python -u tools/tune_route.py "$@" > $O/${T}_B$i.json 2>&1 || { tail $O/${T}_B$i.json; exit 1; }
  echo "B$i $(tail -1 $O/${T}_B$i.json)"
done
