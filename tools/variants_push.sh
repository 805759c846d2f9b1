# Profiling variants (sspp_amd/lib/variants, tools/build_variant.sh) stay out of the gpurun push by
# default (.gpurunignore).  A run that needs them: bash tools/variants_push.sh on; after it: off.
set -e
cd "$(dirname "$0")/.."
LINE=./sspp_amd/lib/variants
case "$1" in
  on)  grep -v "^$LINE\$" .gpurunignore > .gpurunignore.tmp && mv .gpurunignore.tmp .gpurunignore ;;
  off) grep -qx "$LINE" .gpurunignore || echo "$LINE" >> .gpurunignore ;;
  *) echo "usage: $0 on|off" >&2; exit 2 ;;
esac
grep -c "^$LINE\$" .gpurunignore >/dev/null && echo "variants: not pushed" || echo "variants: pushed"
