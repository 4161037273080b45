#!/bin/bash
# Rebuilds oz_gram_kernel<0> of commit 32e45ae (the manual A-load waits that faulted on the GPU and
# were reverted by 632ee2d) and writes tests/isa/reverted_manual_a.s: the excerpt from the last
# step's inline-asm A loads to the first epilogue instructions that reuse their registers.
# The full-kernel check of that build: python tools/isa_vmem_check.py /tmp/isa_rev/gram.s
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/isa_rev
rm -rf "$W" && mkdir -p "$W"
git -C "$ROOT" worktree add -f "$W/wt" 32e45ae >/dev/null
trap 'git -C "$ROOT" worktree remove --force "$W/wt" >/dev/null 2>&1 || true' EXIT
(cd "$W/wt/oaxaca-blinder-rs_amd/csrc" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c ob_gram_i8.hip -o "$W/gram.o")
SYM=_ZN12_GLOBAL__N_114oz_gram_kernelILi0EEEvNS_6OzArgsE
python3 - "$W" <<PY
import sys; sys.path.insert(0, "$ROOT/tools")
import isa_vmem_check as C
print(C.extract_gfx950(sys.argv[1] + "/gram.o", sys.argv[1]))
PY
/opt/rocm/lib/llvm/bin/llvm-objdump -d --mcpu=gfx950 --disassemble-symbols=$SYM "$W/co0.elf" > "$W/gram.s"
{
  echo "; oz_gram_kernel<0> of commit 32e45ae (manual A-load waits, reverted by 632ee2d), gfx950,"
  echo "; llvm-objdump -d --mcpu=gfx950: the last step's A-fragment loads (inline asm, untracked) and the"
  echo "; first instructions after the loop, which reuse v42 and v114 while those loads are in flight."
  echo "; Regenerate: tools/isa_reverted_excerpt.sh"
  grep -m1 "^[0-9a-f]* <" "$W/gram.s"
  awk '/26E44:/,/26F48:/' "$W/gram.s"
} > "$ROOT/tests/isa/reverted_manual_a.s"
python3 "$ROOT/tools/isa_vmem_check.py" "$W/gram.s" | awk '{print $1}' | sort | uniq -c || true
