# Build libbfz.so from a source revision with extra compile definitions, into
# zkvm-brainfuck_amd/variants/libbfz_<name>.so (for scripts/ab_bench.sh):
#   bash scripts/build_variant.sh <name> [<git rev>|WORKTREE] [-DFLAG=value ...]
# The scratch tree lives under .scratch/ inside the repository (git- and gpurun-ignored).
set -e
name=$1; shift
rev=${1:-WORKTREE}; shift || true
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$root/.scratch/variant_$name
rm -rf $tmp && mkdir -p $tmp/zkvm-brainfuck_amd
if [ "$rev" = "WORKTREE" ]; then
  cp -r $root/include $tmp/
  cp -r $root/zkvm-brainfuck_amd/csrc $root/zkvm-brainfuck_amd/bfz $root/zkvm-brainfuck_amd/Makefile $tmp/zkvm-brainfuck_amd/
else
  git -C $root archive $rev include zkvm-brainfuck_amd/csrc zkvm-brainfuck_amd/bfz zkvm-brainfuck_amd/Makefile | tar -x -C $tmp
fi
make -s -C $tmp/zkvm-brainfuck_amd -j16 CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-pass-failed $*" libbfz.so
mkdir -p $root/zkvm-brainfuck_amd/variants
cp $tmp/zkvm-brainfuck_amd/libbfz.so $root/zkvm-brainfuck_amd/variants/libbfz_$name.so
rm -rf $tmp
