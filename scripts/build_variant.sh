# Build libbfz.so from the current sources with extra compile definitions, into
# zkvm-brainfuck_amd/variants/libbfz_<name>.so (for scripts/ab_bench.sh):
#   bash scripts/build_variant.sh a -DBFZ_TILE_DIRECT=0
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=/tmp/bfz_variant_$name
rm -rf $tmp && mkdir -p $tmp/zkvm-brainfuck_amd
cp -r $root/include $tmp/
cp -r $root/zkvm-brainfuck_amd/csrc $root/zkvm-brainfuck_amd/bfz $root/zkvm-brainfuck_amd/Makefile $tmp/zkvm-brainfuck_amd/
make -s -C $tmp/zkvm-brainfuck_amd -j8 CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-pass-failed $*" libbfz.so
mkdir -p $root/zkvm-brainfuck_amd/variants
cp $tmp/zkvm-brainfuck_amd/libbfz.so $root/zkvm-brainfuck_amd/variants/libbfz_$name.so
rm -rf $tmp
