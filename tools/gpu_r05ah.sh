# the whole -m gpu suite twice on one box (queue cap 10), then the default bench line
set -u
KEEP_GOING=1 TESTS_TAG=_1 bash tools/gpu.sh r05ah smoke tests
KEEP_GOING=1 TESTS_TAG=_2 bash tools/gpu.sh r05ah tests bench:c2
