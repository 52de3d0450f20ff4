# Round 3, call 8: c2 N = 1 fell from 1617 it/s (round 2) to 1368: bench the product library of
# each round-3 commit (worktrees under _bisect/, each with its own bench.py) on one box
set -u
O=gpurun_out/r03h
mkdir -p $O
run() {  # dir label
  (cd $1 && timeout -k 10 200 python -u bench.py --config c2 --steps 300 --warmup 30 --no-cpu-baseline) > $O/$2.log 2>&1 || exit $?
  grep '^{' $O/$2.log > $O/$2.json
  echo "$2 $(python3 -c "import json;d=json.load(open('$O/$2.json'));print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
}
run . head
for c in b72e083 ef21cc4 5e24486 6e97eab 1a3da88; do run _bisect/$c $c; done
run . head2
