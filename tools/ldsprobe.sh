set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'orb-slam-system_amd')
import orbx, numpy as np
from orbx import synth
ex=orbx.Extractor(1200,1.2,8,20,7)
k,d=ex.extract(synth.frame(752,480,50))
print('ok',len(k))
"
