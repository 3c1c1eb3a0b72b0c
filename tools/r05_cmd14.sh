#!/bin/bash
# VLC subtraction probes (kernel trace)
R=${GRAFT_REPO_ROOT:-$(pwd)}
CONTENTS="survey" bash $R/tools/vlc_prof.sh abtest/lib_vlc3.so abtest/lib_vprobe1.so abtest/lib_vprobe2.so abtest/lib_vprobe3.so
