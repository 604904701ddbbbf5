set -u
O=gpurun_out/r03_st; mkdir -p $O
timeout -k 10 200 python -u tools/team_stamps.py --rank 1 > $O/stamps_r1.log 2>&1 || exit 1
for g in 4 16; do SPF_MSBFS_TEAM=$g timeout -k 10 200 python -u tools/emulate_ranks.py --worlds 8 > $O/emu_g$g.log 2>&1 || exit 1; done
SPF_MSBFS_TEAM=0 timeout -k 10 200 python -u tools/emulate_ranks.py --worlds 4,8 > $O/emu_noteam.log 2>&1 || exit 1
cat $O/stamps_r1.log; cut -c1-200 $O/emu_g4.log $O/emu_g16.log $O/emu_noteam.log
