#!/bin/bash
# Instruction count + registers of the Homing step kernels (device asm), no GPU needed.
cd "$(dirname "$0")/../swarmacb-isaaclab_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -DSWARM_MISSION_ID=${MISSION:-2} $EXTRA \
  -I../../build/obj/gen --cuda-device-only -S -o /tmp/cs.s swarm_mission.hip -Rpass-analysis=kernel-resource-usage 2> /tmp/cs_res.txt || exit 1
python3 - <<'PY'
import re
s = open('/tmp/cs.s').read()
res = open('/tmp/cs_res.txt').read()
for name in re.findall(r'^(_ZN5swarm11step_kernelI\w+):', s, re.M):
    if 'Lb0ELi20E' not in name: continue
    if not re.search(r'step_kernelILi\dELi0E', name): continue
    start = s.index(name + ':'); end = s.index('.Lfunc_end', start)
    n = sum(1 for l in s[start:end].split('\n') if l.startswith('\t') and not l.startswith('\t.') and not l.startswith('\t;'))
    m = re.search(re.escape(name) + r'.*?VGPRs: (\d+).*?ScratchSize \[bytes/lane\]: (\d+).*?SGPRs Spill: (\d+).*?VGPRs Spill: (\d+)', res, re.S)
    print(name[23:50], 'insts', n, 'vgpr/scratch/sgpr-spill/vgpr-spill', m.groups() if m else None)
PY
