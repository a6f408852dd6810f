import gzip, json, sys, collections
for fn in sys.argv[1:]:
    d = json.load(gzip.open(fn, 'rt'))
    tid = d['tid']; names = {v: k for k, v in tid.items()}
    idle = tid['idle']
    tr = d['trace']
    evs = collections.Counter(r[1] for r in tr)
    # request starts: WAKE of idle slot
    wakes = [r for r in tr if r[1] == 'WAKE' and r[3] == idle]
    sw_in = [r for r in tr if r[1] == 'SWITCH' and r[4] == idle]
    sleeps = [r for r in tr if r[1] == 'SLEEP' and r[3] == idle]
    # group wakes into bursts (gap > 200us)
    bursts = []
    for r in wakes:
        if not bursts or r[0] - bursts[-1][-1][0] > 200000:
            bursts.append([r])
        else:
            bursts[-1].append(r)
    waits = []
    j = 0
    for b in bursts:
        t0 = b[0][0]
        while j < len(sw_in) and sw_in[j][0] < t0:
            j += 1
        if j < len(sw_in):
            waits.append((sw_in[j][0] - t0) / 1e6)
    waits.sort()
    def p(q): return waits[min(len(waits)-1, int(q*(len(waits)-1)))] if waits else None
    lat = sorted(d['lat_ms'])
    pl = lambda q: lat[min(len(lat)-1, int(q*(len(lat)-1)))] if lat else None
    span = (tr[-1][0] - tr[0][0]) / 1e6 if tr else 0
    print(fn.split('/')[-1], 'agg %.4f' % d['aggregate'], 'span_ms %.0f' % span, 'bursts', len(bursts),
          'wait->switch p50/p99/max ms', p(0.5), p(0.99), waits[-1] if waits else None,
          'lat p50/p99/max', pl(0.5), pl(0.99), lat[-1] if lat else None)
    print('   events', dict(evs))
    e = d['engine']
    print('   run_share', e.get('run_share'), 'tslice', e.get('mean_tslice_us'))
