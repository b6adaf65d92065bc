# Writes .source_head (the commit the working tree's library sources were
# committed as; "+dirty" if they differ from it) before a gpurun call, for
# tools/source_stamp.py on the GPU box, which gets the tree without .git.
cd "$(dirname "$0")/.." && h=$(git rev-parse --short=12 HEAD) && \
  { git diff --quiet HEAD -- go-dsp_amd/csrc include && echo "$h" || echo "$h+dirty"; } > .source_head
