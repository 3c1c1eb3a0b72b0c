#!/bin/bash
# k_inter_mbg: +640 dependent VALU per wave (2-clock add, 4-clock alignbyte) -- how VALU-bound is it
R=${GRAFT_REPO_ROOT:-$(pwd)}
CONTENTS="survey" bash $R/tools/inter_prof.sh abtest/lib_base.so abtest/lib_ivadd640.so abtest/lib_ivalign640.so abtest/lib_base.so
