#!/bin/bash
# evidence at head (after the VLC and bench changes): GPU suite, smoke, the
# driver's bench command, rocprof timed region
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=r05f bash $R/tools/r05_evidence.sh || exit 1
echo evidence-done
