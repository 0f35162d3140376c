set -uo pipefail
for spec in ${SPECS:-"vi_st_tail=0,vi_st_faces=1" "vi_st_tail=1,vi_st_faces=1" "vi_st_tail=1,vi_st_faces=0" "vi_st_tail=0,vi_st_faces=0"}; do
  tag=$(echo $spec | tr ',=' '__')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG:-r05n}_$tag -o run --output-format csv -- python3 tools/spmv_kernels.py --grid 256 --sets "$spec" --iters 50 > gpurun_out/${TAG:-r05n}_$tag.log 2>&1 || exit $?
done
