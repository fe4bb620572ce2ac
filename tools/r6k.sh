bash tools/profile_round.sh r06 sf100 q3 > gpurun_out/prof_r06_2.log 2>&1; echo rc=$? >> gpurun_out/prof_r06_2.log
