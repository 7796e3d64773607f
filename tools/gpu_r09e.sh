#!/bin/bash
# round 6: records per lane per group of the concat LDS walk (RPL 2 shipped, 4, 1): library A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_lib_ab.sh r09e_ab 3 "" tools/ab/libgatx_base.so tools/ab/libgatx_rpl4.so tools/ab/libgatx_rpl1.so
