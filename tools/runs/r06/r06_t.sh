#!/bin/bash
# Round 6: the C3 write set three ways plus the check fields alone (2 x 2 B per
# frame), no reads -- do partial sectors write back cheaper than whole ones?
set -o pipefail
O=gpurun_out/${R06_OUT:-r06t}
mkdir -p $O
KB_ONLY='write|no write-back|FRESH (shipped' timeout -k 10 300 tools/kbench imix 4194304 15 > $O/kbench_imix_fields.log 2>&1 || { tail -20 $O/kbench_imix_fields.log; exit 1; }
KB_BLOCKED=1 KB_ONLY='write' timeout -k 10 300 tools/kbench imix 4194304 15 > $O/kbench_imix_fields_blocked.log 2>&1 || { tail -20 $O/kbench_imix_fields_blocked.log; exit 1; }
cat $O/kbench_imix_fields.log $O/kbench_imix_fields_blocked.log | grep -E "write|compute|IMIX"
