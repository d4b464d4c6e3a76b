import cProfile, pstats, sys, os
sys.argv = ["e2e_batch.py", "32", "0"]
cProfile.run(open("scripts/e2e_batch.py").read(), "/root/repo/gpurun_out/e2e.prof")
