# round-6 closing run: full GPU suite + smoke + default bench line (gpu_full.sh final), then the C4 A/B of the
# nontemporal-store library build (tools/ab/libsuta_nt.so, evidence only)
set -e
bash tools/r6/gpu_full.sh final
bash tools/r6/gpu_env_multi.sh ntab "" "" SUTA_LIB=$PWD/tools/ab/libsuta_nt.so -
