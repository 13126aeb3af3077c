#!/usr/bin/env bash
# Install Otedama (MI355X) from a source checkout: build the gfx950 extension
# in-tree and put an `otedama` launcher on PATH. No network access is needed
# beyond what ROCm + PyTorch already provide.
#
#   ./install.sh [--prefix DIR]        (default: ~/.local)
set -euo pipefail

PREFIX="${HOME}/.local"
while [ $# -gt 0 ]; do
  case "$1" in
    --prefix) PREFIX="$2"; shift 2 ;;
    -h|--help) sed -n '2,8p' "$0"; exit 0 ;;
    *) echo "install.sh: unknown argument $1" >&2; exit 64 ;;
  esac
done

SRC="$(cd "$(dirname "$0")" && pwd)"
PY="${PYTHON:-python3}"

command -v hipcc >/dev/null 2>&1 || [ -x /opt/rocm/bin/hipcc ] || {
  echo "install.sh: ROCm hipcc not found (install ROCm 7.x for gfx950)" >&2; exit 1; }
"$PY" -c "import torch" 2>/dev/null || { echo "install.sh: PyTorch (ROCm build) is required" >&2; exit 1; }

echo "==> building native extension for gfx950"
(cd "$SRC" && "$PY" -m otedama_amd._build)

mkdir -p "$PREFIX/bin"
cat > "$PREFIX/bin/otedama" <<EOF
#!/usr/bin/env bash
export PYTHONPATH="$SRC\${PYTHONPATH:+:\$PYTHONPATH}"
export HSA_ENABLE_IPC_MODE_LEGACY=\${HSA_ENABLE_IPC_MODE_LEGACY:-0}
exec "$PY" -m otedama_amd "\$@"
EOF
chmod 0755 "$PREFIX/bin/otedama"
echo "==> installed $PREFIX/bin/otedama"
"$PREFIX/bin/otedama" version
case ":$PATH:" in *":$PREFIX/bin:"*) ;; *) echo "note: add $PREFIX/bin to PATH" ;; esac
