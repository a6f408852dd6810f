"""gpbsctl: the xl analog (X:tools/libxl/xl_cmdtable.c, xl_cmdimpl.c).

Verbs, options, output formats and error strings follow xl with
Domain -> tenant, VCPU -> slot, CPU -> partition (GPU:XCD:context) and
cpupool -> pool:

    gpbsctl sched-credit [-d <Tenant> [-w[=WEIGHT]|-c[=CAP]]] [-s [-t TSLICE] [-r RATELIMIT]] [-p POOL]
    gpbsctl sched-credit2 [-d <Tenant> [-w[=WEIGHT]]] [-p POOL]
    gpbsctl sched-sedf [-d <Tenant> [-p MS] [-s MS] [-l MS] [-e 0|1] [-w W]] [-c POOL]
    gpbsctl sched-arinc653 [-p POOL] [-f MAJOR_FRAME_US TENANT[:SLOT]=RUNTIME_US ...]
    gpbsctl create NAME [--slots N] [--weight W] [--cap C] [--pool P]
    gpbsctl destroy|pause|unpause TENANT
    gpbsctl list | slot-list [TENANT...] | slot-pin TENANT SLOT|all PARTS|all | slot-set TENANT N
    gpbsctl debug-keys KEYS | dmesg [-c] | top | mon [-i S] | trace [-n N] | perfc [-r|--prom] | lockprof [-r] | info
    gpbsctl watchdog DOMAIN ID TIMEOUT_MS        (SCHEDOP_watchdog: ID 0 allocates, TIMEOUT 0 frees)
    gpbsctl pool-create NAME [--sched S] [--cpus C] | pool-list [-c] [POOL] | pool-destroy POOL
    gpbsctl pool-rename POOL NEW | pool-gpu-add POOL PARTS|node:N | pool-gpu-remove POOL PARTS|node:N
    gpbsctl pool-migrate TENANT POOL | pool-xgmi-split | snapshot PATH | restore PATH
"""
from __future__ import annotations

import argparse
import json
import sys
from typing import List, Optional

from .rpc import DEFAULT_SOCKET, Client, RpcError

RUNSTATE = {0: "r", 1: "-", 2: "b", 3: "p"}


def _err(msg: str) -> None:
    print(msg, file=sys.stderr)


def _dom_row(d):
    print("%-33s %4d %6d %4d" % (d["name"], d["id"], d["weight"], d["cap"]))


def _dom_header():
    print("%-33s %4s %6s %4s" % ("Name", "ID", "Weight", "Cap"))


def _pool_line(c: Client, pool) -> None:
    try:
        p = c.call("pool_params_get", pool=pool)
        print("Cpupool %s: tslice=%dus ratelimit=%dus" % (p["name"], p["tslice_us"], p["ratelimit_us"]))
    except RpcError:
        print("Cpupool %s: [sched params unavailable]" % pool)


def cmd_sched_credit(c: Client, argv: List[str]) -> int:
    ap = argparse.ArgumentParser(prog="gpbsctl sched-credit", add_help=True)
    ap.add_argument("-d", "--domain", "--tenant", dest="dom")
    ap.add_argument("-w", "--weight", type=int)
    ap.add_argument("-c", "--cap", type=int)
    ap.add_argument("-s", "--schedparam", action="store_true")
    ap.add_argument("-t", "--tslice_us", type=int)
    ap.add_argument("-r", "--ratelimit_us", type=int)
    ap.add_argument("-p", "--cpupool", "--pool", dest="pool")
    a = ap.parse_args(argv)
    opt_w, opt_c = a.weight is not None, a.cap is not None
    opt_t, opt_r = a.tslice_us is not None, a.ratelimit_us is not None
    if (a.pool or a.schedparam) and (a.dom or opt_w or opt_c):
        _err("Specifying a cpupool or schedparam is not allowed with domain options.")
        return 1
    if not a.dom and (opt_w or opt_c):
        _err("Must specify a domain.")
        return 1
    if not a.schedparam and (opt_t or opt_r):
        _err("Must specify schedparam to set schedule parameter values.")
        return 1
    if a.schedparam:
        pool = a.pool if a.pool is not None else 0
        try:
            c.call("pool_params_get", pool=pool)
        except RpcError:
            _err("unknown cpupool '%s'" % pool)
            return 3
        if not opt_t and not opt_r:
            _pool_line(c, pool)
            return 0
        try:
            c.call("pool_params_set", pool=pool, tslice_us=a.tslice_us, ratelimit_us=a.ratelimit_us)
        except RpcError as e:
            _err(str(e))
            _err("libxl_sched_credit_params_set failed.")
            return 3
        return 0
    if not a.dom:  # list every pool and its tenants
        pools = c.call("pool_list")
        if a.pool is not None:
            match = [p for p in pools if str(p["id"]) == str(a.pool) or p["name"] == a.pool]
            if not match:
                _err("unknown cpupool '%s'" % a.pool)
                return 3
            pools = match
        doms = c.call("domain_list")
        for p in pools:
            if p["sched"] not in ("credit", "credit-fixed", "credit-classq", "atc"):  # credit2 / sedf: their own verbs
                continue
            _pool_line(c, p["id"])
            _dom_header()
            for d in doms:
                if d["pool"] == p["id"]:
                    _dom_row(d)
        return 0
    try:
        if not opt_w and not opt_c:
            d = c.call("domain_sched_get", domain=a.dom)
            _dom_header()
            _dom_row(d)
            return 0
        c.call("domain_sched_set", domain=a.dom, weight=a.weight if opt_w else -1, cap=a.cap if opt_c else -1)
        return 0
    except RpcError as e:
        _err(str(e))
        if opt_w or opt_c:
            _err("libxl_domain_sched_params_set failed.")
        return 3


def _sched_pools(c: Client, sched: str, pool: Optional[str]):
    """Pools running `sched` (optionally one named pool), or None after an
    error message (sched_domain_output, xl_cmdimpl.c:4739-4790)."""
    pools = c.call("pool_list")
    if pool is not None:
        match = [p for p in pools if str(p["id"]) == str(pool) or p["name"] == pool]
        if not match:
            _err("unknown cpupool '%s'" % pool)
            return None
        pools = match
    return [p for p in pools if p["sched"] == sched]


def cmd_sched_credit2(c: Client, argv: List[str]) -> int:
    """xl sched-credit2 (xl_cmdimpl.c:4932-5005): weight only, no caps."""
    ap = argparse.ArgumentParser(prog="gpbsctl sched-credit2", add_help=True)
    ap.add_argument("-d", "--domain", "--tenant", dest="dom")
    ap.add_argument("-w", "--weight", type=int)
    ap.add_argument("-p", "--cpupool", "--pool", dest="pool")
    a = ap.parse_args(argv)
    if a.pool is not None and (a.dom or a.weight is not None):
        _err("Specifying a cpupool is not allowed with other options.")
        return 1
    if not a.dom and a.weight is not None:
        _err("Must specify a domain.")
        return 1
    hdr = lambda: print("%-33s %4s %6s" % ("Name", "ID", "Weight"))
    row = lambda d: print("%-33s %4d %6d" % (d["name"], d["id"], d["weight"]))
    if not a.dom:
        pools = _sched_pools(c, "credit2", a.pool)
        if pools is None:
            return 3
        doms = c.call("domain_list")
        for p in pools:
            print("Cpupool %s:" % p["name"])
            hdr()
            for d in doms:
                if d["pool"] == p["id"]:
                    row(c.call("domain_sched_ext_get", domain=d["id"]))
        return 0
    try:
        if a.weight is None:
            hdr()
            row(c.call("domain_sched_ext_get", domain=a.dom))
        else:
            c.call("domain_sched_ext_set", domain=a.dom, weight=a.weight)
        return 0
    except RpcError as e:
        _err(str(e))
        if a.weight is not None:
            _err("libxl_domain_sched_params_set failed.")
        return 3


def cmd_sched_arinc653(c: Client, argv: List[str]) -> int:
    """ARINC 653 schedule table (the a653sched_adjust_global put/get that the
    reference exposes through xc_sched_arinc653_schedule_set/get).  Without -f
    prints the table; with -f installs a new one, effective at once."""
    ap = argparse.ArgumentParser(prog="gpbsctl sched-arinc653", add_help=True)
    ap.add_argument("-p", "--cpupool", "--pool", dest="pool")
    ap.add_argument("-f", "--major-frame", dest="major", type=float)
    ap.add_argument("entries", nargs="*", help="TENANT[:SLOT]=RUNTIME_US")
    a = ap.parse_args(argv)
    if a.entries and a.major is None:
        _err("Must specify the major frame (-f) with schedule entries.")
        return 1
    if a.major is not None:
        es = []
        for x in a.entries:
            if "=" not in x:
                _err(f"Bad entry '{x}': expected TENANT[:SLOT]=RUNTIME_US")
                return 1
            who, rt = x.split("=", 1)
            dom, slot = (who.split(":", 1) + ["-1"])[:2] if ":" in who else (who, "-1")
            es.append({"domain": dom, "slot": int(slot), "runtime_us": float(rt)})
        c.call("arinc653_set", pool=a.pool, major_frame_us=a.major, entries=es)
    s = c.call("arinc653_get", pool=a.pool)
    print("Cpupool %s: major_frame=%dus%s" % (s["name"], s["major_frame_us"], "" if s["explicit"] else " (automatic)"))
    print("%-33s %4s %5s %10s" % ("Name", "ID", "Slot", "Runtime_us"))
    for e in s["entries"]:
        print("%-33s %4d %5s %10d" % (e["domain"], e["id"], "all" if e["slot"] < 0 else e["slot"], e["runtime_us"]))
    return 0


def cmd_sched_sedf(c: Client, argv: List[str]) -> int:
    """xl sched-sedf (xl_cmdimpl.c:5007-5110).  Times are in ms, as in xl."""
    ap = argparse.ArgumentParser(prog="gpbsctl sched-sedf", add_help=True)
    ap.add_argument("-d", "--domain", "--tenant", dest="dom")
    ap.add_argument("-p", "--period", type=int)
    ap.add_argument("-s", "--slice", type=int)
    ap.add_argument("-l", "--latency", type=int)
    ap.add_argument("-e", "--extra", type=int)
    ap.add_argument("-w", "--weight", type=int)
    ap.add_argument("-c", "--cpupool", "--pool", dest="pool")
    a = ap.parse_args(argv)
    opts = [x is not None for x in (a.period, a.slice, a.latency, a.extra, a.weight)]
    if a.pool is not None and (a.dom or any(opts)):
        _err("Specifying a cpupool is not allowed with other options.")
        return 1
    if not a.dom and any(opts):
        _err("Must specify a domain.")
        return 1
    if a.weight is not None and (a.period is not None or a.slice is not None):
        _err("Specifying a weight AND period or slice is not allowed.")
    hdr = lambda: print("%-33s %4s %6s %-6s %7s %5s %6s" % ("Name", "ID", "Period", "Slice", "Latency", "Extra",
                                                           "Weight"))
    row = lambda d: print("%-33s %4d %6d %6d %7d %5d %6d" % (d["name"], d["id"], d["period_us"] // 1000,
                                                            d["slice_us"] // 1000, d["latency_us"] // 1000,
                                                            d["extratime"], d["weight"]))
    if not a.dom:
        pools = _sched_pools(c, "sedf", a.pool)
        if pools is None:
            return 3
        doms = c.call("domain_list")
        for p in pools:
            print("Cpupool %s:" % p["name"])
            hdr()
            for d in doms:
                if d["pool"] == p["id"]:
                    row(c.call("domain_sched_ext_get", domain=d["id"]))
        return 0
    try:
        if not any(opts):
            hdr()
            row(c.call("domain_sched_ext_get", domain=a.dom))
            return 0
        cur = c.call("domain_sched_ext_get", domain=a.dom)
        kw = dict(weight=0, period_us=cur["period_us"], slice_us=cur["slice_us"], latency_us=-1, extratime=-1)
        if a.period is not None:
            kw["period_us"] = a.period * 1000
        if a.slice is not None:
            kw["slice_us"] = a.slice * 1000
        if a.latency is not None:
            kw["latency_us"] = a.latency * 1000
        if a.extra is not None:
            kw["extratime"] = a.extra
        if a.weight is not None:
            kw.update(weight=a.weight, period_us=0, slice_us=0)
        elif cur["weight"] and a.period is None and a.slice is None:
            kw.update(weight=cur["weight"], period_us=0, slice_us=0)  # -l / -e on a weight-driven tenant
        c.call("domain_sched_ext_set", domain=a.dom, **kw)
        return 0
    except RpcError as e:
        _err(str(e))
        _err("libxl_domain_sched_params_set failed.")
        return 3


def cmd_list(c: Client, argv) -> int:
    doms = c.call("domain_list")
    print("%-40s %5s %5s %5s %10s %8s %6s" % ("Name", "ID", "Slots", "State", "Time(s)", "Tslice", "Phase"))
    for d in doms:
        st = "p" if d["paused"] else "r"
        print("%-40s %5d %5d %5s %10.1f %6dus %6s" % (d["name"], d["id"], d["slots"], st, d["run_ns"] / 1e9,
                                                    d["tslice_us"], {1: "LOW", 2: "HIGH"}.get(d["phase"], "-")))
    return 0


def cmd_slot_list(c: Client, argv) -> int:
    rows = c.call("slot_list", domains=argv or None)
    print("%-32s %5s %5s %5s %5s %9s %7s %4s" % ("Name", "ID", "SLOT", "PART", "State", "Time(s)", "Credit", "Pri"))
    for r in rows:
        print("%-32s %5d %5d %5d %5s %9.1f %7d %4d" % (r["name"], r["id"], r["slot"], r["cpu"],
                                                      RUNSTATE.get(r["state"], "?"), r["time_s"], r["credit"],
                                                      r["pri"]))
    return 0


def cmd_top(c: Client, argv) -> int:
    t = c.call("top")
    print("%-20s %4s %5s %6s %9s %8s %5s %7s %10s %8s %7s %14s" % (
        "NAME", "ID", "POOL", "SLOTS", "RUN(s)", "TSLICE", "PHASE", "CLASS", "MISSRATE", "CPI", "REPORTS", "VPMU_INST"))
    for r in t["tenants"]:
        print("%-20s %4d %5d %3d/%-2d %9.2f %6dus %5s %7s %10d %8d %7d %14d" % (
            r["name"][:20], r["id"], r["pool"], r["active"], r["slots"], r["run_s"], r["tslice_us"],
            {1: "LOW", 2: "HIGH"}.get(r["phase"], "-"), {0: "compute", 1: "memory"}.get(r.get("class", -1), "-"),
            r["miss_rate"], r["cpi"], r["reports"], r.get("vpmu", {}).get("INST_RETIRED", 0)))
    busy = sum(1 for p in t["partitions"] if not p["idle"])
    print(f"partitions busy: {busy}/{len(t['partitions'])}")
    return 0


def cmd_lockprof(c: Client, argv) -> int:
    """xenlockprof output shape: lock count(time), block count(time)."""
    p = c.call("lockprof", reset="-r" in argv)
    print("%-32s: lock:%12d(%8.6fs), block:%12d(%8.6fs)" % ("gpbs engine lock", p["lock_cnt"],
                                                            p["time_hold_ns"] / 1e9, p["block_cnt"],
                                                            p["time_block_ns"] / 1e9))
    print("%-32s: max hold %.1fus, max block %.1fus, dispatcher hand-offs %d" % (
        "", p["max_hold_ns"] / 1e3, p["max_block_ns"] / 1e3, p["handoffs"]))
    return 0


def cmd_mon(c: Client, argv) -> int:
    """xenmon: gotten / waited / blocked per tenant over an interval."""
    ap = argparse.ArgumentParser(prog="gpbsctl mon")
    ap.add_argument("-i", "--interval", type=float, default=1.0)
    a = ap.parse_args(argv)
    c.call("mon", reset=True)
    import time as _t
    _t.sleep(max(0.0, a.interval))
    m = c.call("mon")
    print("interval %.3fs" % m["interval_s"])
    print("%-24s %4s %5s %9s %9s %9s %10s" % ("Name", "ID", "Slots", "Gotten%", "Waited%", "Blocked%", "Execs/s"))
    for r in m["tenants"]:
        print("%-24s %4d %5d %9.2f %9.2f %9.2f %10.1f" % (r["name"][:24], r["id"], r["slots"], r["gotten_pct"],
                                                        r["waited_pct"], r["blocked_pct"], r["execs_per_s"]))
    return 0


def cmd_pool_list(c: Client, argv) -> int:
    ap = argparse.ArgumentParser(prog="gpbsctl pool-list")
    ap.add_argument("-c", "--cpus", action="store_true")
    ap.add_argument("pool", nargs="?")
    a = ap.parse_args(argv)
    pools = c.call("pool_list")
    if a.pool is not None:
        pools = [p for p in pools if p["name"] == a.pool or str(p["id"]) == a.pool]
        if not pools:
            _err("unknown cpupool '%s'" % a.pool)
            return 1
    if a.cpus:
        print("%-32s %s" % ("Name", "CPU list"))
        for p in pools:
            print("%-32s %s" % (p["name"], ",".join(str(x) for x in p["cpus"])))
    else:
        print("%-32s %6s %-10s %6s %7s" % ("Name", "CPUs", "Sched", "Active", "Domain count"))
        for p in pools:
            print("%-32s %6d %-10s %6s %7d" % (p["name"], len(p["cpus"]), p["sched"], "y", p["n_tenants"]))
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    sock = DEFAULT_SOCKET
    if argv[:1] == ["--socket"] and len(argv) > 1:
        sock = argv[1]
        argv = argv[2:]
    if not argv or argv[0] in ("-h", "--help", "help"):
        print(__doc__)
        return 0
    cmd, rest = argv[0], argv[1:]
    try:
        c = Client(sock)
    except OSError as e:
        _err(f"cannot connect to gpbsd at {sock}: {e}")
        return 2
    try:
        if cmd == "sched-credit":
            return cmd_sched_credit(c, rest)
        if cmd == "sched-credit2":
            return cmd_sched_credit2(c, rest)
        if cmd == "sched-sedf":
            return cmd_sched_sedf(c, rest)
        if cmd == "sched-arinc653":
            return cmd_sched_arinc653(c, rest)
        if cmd == "list":
            return cmd_list(c, rest)
        if cmd in ("slot-list", "vcpu-list"):
            return cmd_slot_list(c, rest)
        if cmd == "top":
            return cmd_top(c, rest)
        if cmd in ("pool-list", "cpupool-list"):
            return cmd_pool_list(c, rest)
        simple = {
            "create": lambda r: c.call("create", **_kv(r, ("name",), dict(slots=int, weight=int, cap=int, pool=str))),
            "destroy": lambda r: c.call("destroy", domain=r[0]),
            "pause": lambda r: c.call("pause", domain=r[0]),
            "unpause": lambda r: c.call("unpause", domain=r[0]),
            "slot-pin": lambda r: c.call("slot_pin", domain=r[0], slot=r[1], cpus=r[2]),
            "vcpu-pin": lambda r: c.call("slot_pin", domain=r[0], slot=r[1], cpus=r[2]),
            "slot-set": lambda r: c.call("slot_set", domain=r[0], n=int(r[1])),
            "vcpu-set": lambda r: c.call("slot_set", domain=r[0], n=int(r[1])),
            "pool-create": lambda r: c.call("pool_create", **_kv(r, ("name",), dict(sched=str, cpus=str))),
            "cpupool-create": lambda r: c.call("pool_create", **_kv(r, ("name",), dict(sched=str, cpus=str))),
            "pool-destroy": lambda r: c.call("pool_destroy", pool=r[0]),
            "cpupool-destroy": lambda r: c.call("pool_destroy", pool=r[0]),
            "pool-rename": lambda r: c.call("pool_rename", pool=r[0], name=r[1]),
            "cpupool-rename": lambda r: c.call("pool_rename", pool=r[0], name=r[1]),
            "pool-gpu-add": lambda r: c.call("pool_cpu_add", pool=r[0], cpu=r[1]),
            "cpupool-cpu-add": lambda r: c.call("pool_cpu_add", pool=r[0], cpu=r[1]),
            "pool-gpu-remove": lambda r: c.call("pool_cpu_remove", pool=r[0], cpu=r[1]),
            "cpupool-cpu-remove": lambda r: c.call("pool_cpu_remove", pool=r[0], cpu=r[1]),
            "pool-migrate": lambda r: c.call("pool_migrate", domain=r[0], pool=r[1]),
            "cpupool-migrate": lambda r: c.call("pool_migrate", domain=r[0], pool=r[1]),
            "pool-xgmi-split": lambda r: c.call("pool_xgmi_split"),
            "cpupool-numa-split": lambda r: c.call("pool_xgmi_split"),
            "snapshot": lambda r: c.call("snapshot", path=r[0] if r else None),
            "restore": lambda r: c.call("restore", path=r[0]),
            "info": lambda r: c.call("info"),
        }
        if cmd == "debug-keys":
            if not rest:
                _err("'gpbsctl debug-keys' requires one argument.")
                return 1
            out = c.call("debug_keys", keys=rest[0])
            sys.stdout.write(out)
            return 0
        if cmd == "dmesg":
            sys.stdout.write(c.call("dmesg", clear="-c" in rest))
            return 0
        if cmd == "trace":
            n = int(rest[rest.index("-n") + 1]) if "-n" in rest else 4096
            for t, ev, cpu, a in c.call("trace", max_records=n, from_start=True):
                print(f"{t / 1e9:14.6f} cpu{cpu:<3d} {ev:<10s} {a[0]:>10d} {a[1]:>10d} {a[2]:>10d} {a[3]:>10d}")
            return 0
        if cmd == "perfc":
            if "--prom" in rest:
                sys.stdout.write(c.call("perfc_prom"))
                return 0
            for k, v in c.call("perfc", reset="-r" in rest).items():
                print(f"{k:<28s} {v}")
            return 0
        if cmd == "lockprof":
            return cmd_lockprof(c, rest)
        if cmd == "mon":
            return cmd_mon(c, rest)
        if cmd == "watchdog":
            if len(rest) < 3:
                _err("'gpbsctl watchdog' requires <Domain> <ID> <TimeoutMs>.")
                return 1
            print(c.call("watchdog", domain=rest[0], id=int(rest[1]), timeout_ms=int(rest[2])))
            return 0
        if cmd in simple:
            res = simple[cmd](rest)
            if isinstance(res, (dict, list)):
                print(json.dumps(res, indent=1))
            elif cmd == "create":
                print(res)
            return 0
        _err(f"command '{cmd}' not implemented")
        return 1
    except IndexError:
        _err(f"'gpbsctl {cmd}' requires more arguments.")
        return 1
    except RpcError as e:
        _err(str(e))
        return 3
    finally:
        c.close()


def _kv(rest, positional, types):
    """Parse 'NAME --key val' style arguments."""
    ap = argparse.ArgumentParser(add_help=False)
    for p in positional:
        ap.add_argument(p)
    for k, ty in types.items():
        ap.add_argument("--" + k, type=ty, default=None)
    a = vars(ap.parse_args(rest))
    return {k: v for k, v in a.items() if v is not None}


if __name__ == "__main__":
    sys.exit(main())
