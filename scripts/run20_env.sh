#!/bin/bash
# run20_timeline.py --brief under each environment setting given ("-" = none, else VAR=v[,VAR=v])
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for setting in "$@"; do
  envs=()
  [ "$setting" != "-" ] && IFS=, read -ra envs <<< "$setting"
  echo "== $setting"
  env "${envs[@]}" timeout -k 10 120 python -u $R/scripts/run20_timeline.py --brief || { echo "failed: $setting"; exit 1; }
done
