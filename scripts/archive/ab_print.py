import json, sys
for n in sys.argv[1:]:
    r = json.load(open("gpurun_out/ab/%s.json" % n))
    print(n, r["roofline"]["copy_ceiling"]["GBps"], r["roofline"]["frac"])
