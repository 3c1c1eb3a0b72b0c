#!/bin/bash
# k_motion: +64 dependent VALU per MB (2-clock add, 4-clock alignbyte) -- how VALU-bound is it
R=${GRAFT_REPO_ROOT:-$(pwd)}
CONTENTS="survey synth" REPS=15 bash $R/tools/me_prof.sh abtest/lib_base.so abtest/lib_vadd64.so abtest/lib_valign64.so abtest/lib_base.so
