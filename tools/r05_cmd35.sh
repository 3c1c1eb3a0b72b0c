#!/bin/bash
# evidence at head (k_motion micro-optimisations): GPU suite, smoke, the
# driver's bench command, rocprof timed region; PMC passes for survey and synth
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=r05j bash $R/tools/r05_evidence.sh || exit 1

echo evidence-done
