# A/B base: group_hash.hip as committed at HEAD (run from the variant's csrc copy)
import subprocess
src = subprocess.run(["git", "-C", "/root/repo", "show", "HEAD:spacedrive_amd/csrc/group_hash.hip"],
                     check=True, capture_output=True, text=True).stdout
open("group_hash.hip", "w").write(src)
