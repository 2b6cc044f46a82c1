set -u
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [[ $rc -gt 1 ]] && exit $rc
timeout -k 10 600 python scripts/sweep.py --n 65536,1048576,16777216 --ifid "block=1024,pf=1,tab=2,dma=1,np=1,bpc=1" --zero "block=1024,pf=1,tab=2,dma=1,np=1,bpc=1;block=1024,pf=1,tab=4,dma=1,np=1;block=1024,pf=1,tab=4,dma=1,np=2;block=1024,pf=2,tab=2,dma=1,np=1,bpc=1;block=768,pf=1,tab=2,dma=1,np=1,bpc=2;block=1024,pf=1,tab=2,dma=1,np=1,bpc=2" > gpurun_out/sweep_d.log 2>&1 || exit $?
cat gpurun_out/sweep_d.log
