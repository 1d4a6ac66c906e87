# one GPU call: A* 2D traffic attribution across engines / LDS heap shares
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 bash tools/traffic_probe.sh mq32:2:1:8192:32 mq8:2:1:2048:8 mq4:2:1:1024:4 w18:0:0:768:18 w4:0:0:1024:4 > gpurun_out/r3_traffic.log 2>&1
