#!/usr/bin/env bash
# Apply the libnxec C++ surface overlay to a Nexoedge source tree
# (INTEGRATION.md Option B; the actions are tools/overlay_manifest.txt).
#
#   tools/overlay_reference.sh <nexoedge tree> [NXEC_ROOT]
#
# <nexoedge tree> is a writable copy of the Nexoedge sources (the directory
# holding CMakeLists.txt and src/).  NXEC_ROOT defaults to this repository.
# The script is idempotent: a tree already overlaid is left as it is (a
# marker file records the NXEC_ROOT it was overlaid with).  After it, the
# usual cmake build links every target against
# <NXEC_ROOT>/nexoedge_amd/lib/libnxec.so (build it with `make` first) and the
# reference's RSCode / CodingOptions sources are gone.
set -euo pipefail
set -f  # manifest items hold glob characters (?<probe>=...)

tree=${1:?usage: overlay_reference.sh <nexoedge tree> [NXEC_ROOT]}
here=$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)
root=$(cd "${2:-$here}" && pwd)
manifest="$here/tools/overlay_manifest.txt"
tree=$(cd "$tree" && pwd)

[ -f "$tree/src/common/coding/rs.hh" ] && [ -f "$tree/CMakeLists.txt" ] \
  || { echo "overlay: $tree does not look like a Nexoedge tree (no src/common/coding/rs.hh)" >&2; exit 2; }
[ -f "$root/nexoedge_amd/csrc/coding/rs.hh" ] \
  || { echo "overlay: $root is not an nxec checkout" >&2; exit 2; }
marker="$tree/.nxec_overlay"
if [ -f "$marker" ]; then
  echo "overlay: $tree already overlaid ($(head -1 "$marker"))"
  exit 0
fi

trim() { local s=$1; s=${s#"${s%%[![:space:]]*}"}; s=${s%"${s##*[![:space:]]}"}; printf '%s' "$s"; }

# forwarder <path> <guard> <libnxec header> <prelude...>
forwarder() {
  local path=$1 guard=$2 header=$3 prelude=$4 item probe inc
  {
    echo "// NXEC-OVERLAY: replaced by tools/overlay_reference.sh (tools/overlay_manifest.txt)."
    echo "// The reference's $path now forwards to libnxec's C++ coding surface,"
    echo "// nexoedge_amd/csrc/coding/$header, after including what the original included."
    echo "#ifndef $guard"
    echo "#define $guard"
    for item in $prelude; do
      if [ "${item:0:1}" = "?" ]; then
        probe=${item%%=*}; probe=${probe:1}; inc=${item#*=}
        echo "#if __has_include($probe)"
        echo "#include $inc"
        echo "#endif"
      else
        echo "#include $item"
      fi
    done
    echo "#include <nexoedge_amd/csrc/coding/$header>"
    echo "#endif  // $guard"
  } > "$tree/$path"
}

applied=()
while IFS= read -r line; do
  case "$line" in ''|'#'*) continue;; esac
  IFS='|' read -r action path f3 f4 f5 <<< "$line"
  action=$(trim "$action"); path=$(trim "$path"); f3=$(trim "${f3:-}"); f4=$(trim "${f4:-}"); f5=$(trim "${f5:-}")
  case "$action" in
    forward)
      [ -f "$tree/$path" ] || { echo "overlay: missing $path" >&2; exit 3; }
      forwarder "$path" "$f3" "$f4" "$f5" ;;
    keep)
      [ -f "$tree/$path" ] || { echo "overlay: missing $path" >&2; exit 3; } ;;
    remove)
      rm -f "$tree/$path" ;;
    add)
      cp "$root/$f3" "$tree/$path" ;;
    patch)
      case "$path" in
        CMakeLists.txt)
          # after the reference's own include_directories, before add_subdirectory
          python3 - "$tree/$path" "$root" <<'EOF'
import re, sys
p, root = sys.argv[1], sys.argv[2]
s = open(p).read()
block = (
    "\n# ---- NXEC-OVERLAY (tools/overlay_reference.sh): RS coding on MI355X through libnxec\n"
    f'set ( NXEC_ROOT "{root}" CACHE PATH "nxec checkout (libnxec.so + headers)" )\n'
    "include_directories ( BEFORE ${NXEC_ROOT} ${NXEC_ROOT}/include )\n"
    "link_libraries ( ${NXEC_ROOT}/nexoedge_amd/lib/libnxec.so )\n"
)
anchor = re.search(r"^add_subdirectory\s*\(\s*src/common\s*\)", s, re.M)
if not anchor:
    sys.exit("overlay: no add_subdirectory( src/common ) in CMakeLists.txt")
s = s[: anchor.start()] + block.lstrip("\n") + "\n" + s[anchor.start():]
open(p, "w").write(s)
EOF
          ;;
        src/common/CMakeLists.txt)
          python3 - "$tree/$path" <<'EOF'
import re, sys
p = sys.argv[1]
s = open(p).read()
s2 = re.sub(r"add_dependencies\(\s*ncloud_code\s+google-log\s+isa-l\s*\)",
            "add_dependencies( ncloud_code google-log )  # NXEC-OVERLAY: no isa-l", s)
s2 = re.sub(r"target_link_libraries\(\s*ncloud_code\s+isal\s+",
            "target_link_libraries( ncloud_code ${NXEC_ROOT}/nexoedge_amd/lib/libnxec.so ", s2)
if s2 == s or "isal" in re.sub(r"#.*", "", s2.split("ncloud_config")[0]):
    sys.exit("overlay: src/common/CMakeLists.txt: ncloud_code's isal lines not found")
open(p, "w").write(s2)
EOF
          ;;
        *) echo "overlay: no patch rule for $path" >&2; exit 3 ;;
      esac ;;
    *) echo "overlay: unknown action '$action'" >&2; exit 3 ;;
  esac
  applied+=("$action $path")
done < "$manifest"

{ echo "NXEC_ROOT=$root"; printf '%s\n' "${applied[@]}"; } > "$marker"
echo "overlay: applied ${#applied[@]} actions to $tree (NXEC_ROOT=$root)"
