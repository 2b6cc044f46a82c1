set -u
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python scripts/sweep.py --rounds 3 --n 1048576,16777216 --ifid "block=1024,pf=1,tab=2,dma=1,np=1,bpc=1" --zero "block=1024,pf=1,tab=2,dma=1,np=1,bpc=1;block=1024,pf=1,tab=2,dma=1,np=1,bpc=2;block=768,pf=1,tab=2,dma=1,np=1,bpc=2;block=512,pf=1,tab=2,dma=1,np=1,bpc=2;block=1024,pf=1,tab=4,dma=1,np=1" > gpurun_out/sweep_e.log 2>&1 || exit $?
cat gpurun_out/sweep_e.log
