# A/B of lib_alt (baseline build) and lib (candidate): the GPU tests named by AB_TESTS on each, then the bench
# alternated twice (tools/gpu_ab.sh).   AB_TESTS="tests/test_gpu_fim2d.py ..." bash tools/gpu_ab_libs.sh [bench args]
export TMPDIR=/tmp
AB_TESTS="${AB_TESTS:-tests/test_gpu_fim2d.py tests/test_gpu_fim3d.py}" LIBS="lib_alt lib" bash tools/gpu_ab.sh "$@"
