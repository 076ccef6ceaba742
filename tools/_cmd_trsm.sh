cd $GRAFT_REPO_ROOT && bash tools/blk_ab.sh trsm "BRD_S1_BLOCKED=1;BRD_LIB=tools/diaglib/trsmfree.so" 2>&1 | grep -E "==|cqr|prep"
