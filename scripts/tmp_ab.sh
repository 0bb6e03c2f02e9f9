cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ENVS="MR_TR_AR=1 MR_LO_POP=0;MR_TR_AR=1;MR_TR_AR=8;MR_TR_AR=16;MR_TR_AR=16 MR_LO_ROT=0;MR_TR_AR=16 MR_LO_POP=0" bash scripts/r05.sh ar envab || exit 1
ENVS="MR_TR_AR=1 MR_LO_POP=0;MR_TR_AR=16;MR_TR_AR=16 MR_LO_ROT=0" bash scripts/r05.sh ar pmcenv
