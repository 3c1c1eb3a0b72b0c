#!/bin/bash
# evidence at head: GPU suite, smoke, the driver's bench command, rocprof timed
# region; then the PMC passes for survey and synth (no stress contents)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=r05d bash $R/tools/r05_evidence.sh || exit 1
STRESS="" bash $R/tools/pmc_bench.sh || exit 1
echo evidence-done
