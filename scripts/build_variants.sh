# Measurement builds for A/B timing: each "name:flags[:source]" compiles keydeps.hip (or the given
# copy of it, e.g. a previous revision) with the extra flags and links libaccord_deps_<name>.so from
# the other objects of the current build (run `make` first).
set -e
cd "$(dirname "$0")/../cassandra-accord_amd"
for spec in "$@"; do
  IFS=: read -r name flags src <<< "$spec"
  src=${src:-csrc/keydeps.hip}
  mkdir -p build/var_$name
  [ "$src" != csrc/keydeps.hip ] && cp "$src" csrc/.var_$name.hip && src=csrc/.var_$name.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $flags -c $src -o build/var_$name/keydeps.o &
done
wait
rm -f csrc/.var_*.hip
for spec in "$@"; do
  IFS=: read -r name flags src <<< "$spec"
  objs=$(ls build/*.o | grep -v '/keydeps.o$')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libaccord_deps_$name.so build/var_$name/keydeps.o $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
ls -la libaccord_deps_*.so
