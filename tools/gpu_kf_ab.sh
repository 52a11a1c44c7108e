# key frame (k_flow) of the current build against alternative builds, twice in rotation
# usage: bash tools/gpu_kf_ab.sh other.so [more.so ...]
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for lib in "" "$@"; do
    if [ -n "$lib" ]; then export AV1R_LIB=$lib; else unset AV1R_LIB; fi
    echo "lib ${lib:-current}"
    timeout -k 10 120 python3 -u tools/keyframe_time.py 10 k_flow | head -1 || exit 1
  done
done
