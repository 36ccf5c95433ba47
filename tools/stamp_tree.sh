#!/bin/bash
# Record the git head (+ "-dirty" when the working tree has changes) of the
# tree a gpurun call is about to measure: tools/prof_summary.py stamps every
# traffic_*.json with it.  Run from the repo root before gpurun.
h=$(git rev-parse --short HEAD)
git diff --quiet HEAD -- . ':!profiles' ':!gpurun_out' || h="$h-dirty"
echo "$h" > .tree_stamp
