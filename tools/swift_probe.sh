#!/bin/bash
# SURVEY.md 7 / VERDICT r04 item 1: is there a Swift toolchain on the GPU box?  Prints what it finds;
# when `swift` exists it also builds and tests the swift/ package against libgsm_amd.so.
# Installs nothing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
echo "date: $(date -u +%FT%TZ)  host: $(hostname)  user: $(id -un)"
echo "uname: $(uname -srm)"
[ -r /etc/os-release ] && grep -E '^(PRETTY_NAME|VERSION_ID)=' /etc/os-release
echo "--- command -v swift swiftc swift-build swift-test"
for c in swift swiftc swift-build swift-test; do printf '%-12s %s\n' "$c" "$(command -v $c || echo '(not found)')"; done
echo "--- swift --version"
swift --version 2>&1 || echo "(rc=$?)"
echo "--- search of the usual install prefixes for a swift driver"
for d in /usr/bin /usr/local/bin /opt /usr/share /usr/local /root/.swiftpm /usr/libexec; do
  [ -d "$d" ] && timeout 20 find "$d" -maxdepth 4 -name 'swift*' -type f -perm -u+x 2>/dev/null | head -n 5
done
echo "--- PATH=$PATH"
if command -v swift >/dev/null 2>&1; then
  echo "--- swift build / swift test of swift/ (libgsm_amd.so from gsm-renderer_amd/lib)"
  export LD_LIBRARY_PATH="$PWD/gsm-renderer_amd/lib:/opt/rocm/lib:${LD_LIBRARY_PATH:-}"
  (cd swift && timeout -k 10 600 swift build -Xlinker -L"$PWD/../gsm-renderer_amd/lib" -Xlinker -L/opt/rocm/lib 2>&1 | tail -n 40)
  (cd swift && timeout -k 10 600 swift test -Xlinker -L"$PWD/../gsm-renderer_amd/lib" -Xlinker -L/opt/rocm/lib 2>&1 | tail -n 60)
fi
echo "--- end"
