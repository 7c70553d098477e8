# round-6 closing run: full GPU suite + smoke + default bench line (gpu_full.sh $1), then a C4 A/B of the library in
# tools/ab/$2 against the in-tree one (evidence only)
set -e
bash tools/r6/gpu_full.sh ${1:-final}
if [ -n "$2" ]; then bash tools/r6/gpu_env_multi.sh ${1:-final}_ab "" "" SUTA_LIB=$PWD/tools/ab/$2 -; fi
