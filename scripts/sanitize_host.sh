# Host C++ runtime under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).
# Builds build/san/_C.so (MDT_SANITIZE=1) and runs the CPU tests that drive the
# native runtime (c10d bucket reducer over gloo, trainer replicas, planners).
set -o pipefail
cd "$(dirname "$0")/.."
MDT_SANITIZE=1 python -m multidisttorch_amd._build -j 8 > /dev/null
export LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:print_summary=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export MDT_NATIVE_SO=$PWD/build/san/_C.so
python - <<'PY'
import torch
from multidisttorch_amd.ops import native
C = native.require()
maps = open("/proc/self/maps").read()
assert C.__file__.endswith("build/san/_C.so"), C.__file__
assert "libasan" in maps and "libubsan" in maps
print("sanitized runtime loaded:", C.__file__)
PY
python -m pytest -q -p no:cacheprovider "$@" \
  tests/multiproc/test_multiprocess.py::test_native_and_python_reducer \
  tests/multiproc/test_multiprocess.py::test_trainer_replicas_stay_in_sync \
  tests/multiproc/test_multiprocess.py::test_bucket_autotune_agrees_across_group \
  tests/unit/test_native_host.py
