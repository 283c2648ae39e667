bash tools/gpu_lease.sh exchange --steps 20 --warmup 3 --cpu-sample-reads 0 --cpu-mt-reads 0 --c3-steps 0 > gpurun_out/ex1.txt 2>&1
tail -2 gpurun_out/ex1.txt
bash tools/gpu_lease.sh suite > gpurun_out/suite1.txt 2>&1
tail -15 gpurun_out/suite1.txt
