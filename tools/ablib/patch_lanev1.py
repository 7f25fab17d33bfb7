# the validator as first committed with the lane path (c477d93: no tail cut, one radix
# pass, segment kernels not launched on the lane path) for a same-box A/B
import subprocess
old = subprocess.run(['git', '-C', '/root/repo', 'show', 'c477d93:spacedrive_amd/csrc/checksum.hip'],
                     check=True, capture_output=True, text=True).stdout
open('checksum.hip', 'w').write(old)
