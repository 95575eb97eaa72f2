set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for x in 0 2400 9500 22000; do
  lib=gobeansdb_amd/libqlzx.so; [ $x -ne 0 ] && lib=gobeansdb_amd/libqlzx_occ$x.so
  QLZX_LIB=$lib bash tools/prof.sh occ$x --blocks 262144 --unique 16384 --steps 3 --warmup 1 --no-cpu | grep "k_dec_blocks" | cut -c1-20,140-200 || exit 1
done
