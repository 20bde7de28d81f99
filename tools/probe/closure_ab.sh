# Same-box A/B of two libmaxcover builds on the single-candidate closure (tools/closure_prof.py)
set -u
A=$1; B=$2
for r in 1 2 3; do
  for v in A B; do
    lib=$A; [ "$v" = B ] && lib=$B
    MAXCOVER_LIB=$lib timeout -k 10 200 python tools/closure_prof.py --calls 400 | sed "s/^/$v /" || exit $?
  done
done
