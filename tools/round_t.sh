set -o pipefail
bash tools/sub_probe.sh r02t sub1 1 | tail -3 && bash tools/sub_probe.sh r02t sub2 2 | tail -3 && bash tools/sub_probe.sh r02t sub3 3 | tail -3 && bash tools/ab.sh r02t 4 var/lib_gnw0.so var/lib_gnw1.so | tail -2
