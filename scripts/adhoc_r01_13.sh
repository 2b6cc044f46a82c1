set -u
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python scripts/sweep.py --rounds 4 --n 1048576,16777216 --ifid "block=1024,pf=1,tab=2,dma=1,bpc=1,dyn=0;block=1024,pf=1,tab=2,dma=1,bpc=1,dyn=1" --zero "block=1024,pf=1,tab=2,dma=1,bpc=1,dyn=0;block=1024,pf=1,tab=2,dma=1,bpc=1,dyn=1;block=1024,pf=1,tab=4,dma=1,dyn=1;block=512,pf=1,tab=2,dma=1,bpc=2,dyn=1;block=1024,pf=1,tab=2,dma=1,bpc=2,dyn=1" > gpurun_out/sweep_f.log 2>&1 || exit $?
HFV_KVARIANT="block=1024,pf=1,tab=2,dma=1,bpc=1,dyn=1" timeout -k 10 300 python scripts/stamps.py 1048576,16777216 > gpurun_out/stamps_dyn.log 2>&1 || exit $?
