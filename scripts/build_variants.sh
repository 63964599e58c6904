# Measurement builds for A/B timing: each "name:flags[:source[:object]]" compiles the given source
# (default csrc/keydeps.hip; e.g. a previous revision or an edited copy) with the extra flags as
# build/<object>.o (default keydeps) and links libaccord_deps_<name>.so from it and the other
# objects of the current build (run `make` first).
set -e
cd "$(dirname "$0")/../cassandra-accord_amd"
for spec in "$@"; do
  IFS=: read -r name flags src obj <<< "$spec"
  obj=${obj:-keydeps}; src=${src:-csrc/$obj.hip}
  mkdir -p build/var_$name
  [ "$src" != csrc/$obj.hip ] && cp "$src" csrc/.var_$name.hip && src=csrc/.var_$name.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wall -Wno-unused-function $flags -c $src -o build/var_$name/$obj.o &
done
wait
rm -f csrc/.var_*.hip
for spec in "$@"; do
  IFS=: read -r name flags src obj <<< "$spec"
  obj=${obj:-keydeps}
  objs=$(ls build/*.o | grep -v "/$obj.o\$")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libaccord_deps_$name.so build/var_$name/$obj.o $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
ls -la libaccord_deps_*.so
