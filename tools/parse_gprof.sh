# Host parser flat profile (gprof): the parser's sources and tools/parse_gprof_driver.cpp
# built with -pg into /tmp, run over a 12-frame tools/bsw 1080p_s1 stream three times.
# usage: bash tools/parse_gprof.sh > profiles/<name>.txt   (CPU only)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
D=$(mktemp -d)
python3 -c "
import sys; sys.path.insert(0, '$R/tools/bsw'); import pybsw
open('$D/s.ivf', 'wb').write(pybsw.stream_ivf('1080p_s1', frames=12, seed=0x5EED1000))"
g++ -O2 -pg -std=c++17 -I"$R/include" -I"$R/av1dec_amd/csrc/parse" "$R"/av1dec_amd/csrc/parse/{obu,block,api}.cpp \
    "$R/tools/parse_gprof_driver.cpp" -o "$D/drv" -lpthread
(cd "$D" && ./drv s.ivf 3 && gprof -b -p ./drv gmon.out | head -24)
rm -rf "$D"
