"""cProfile of one SpfSolver.buildRouteDb(me) step of the fabric_lfa_routes
bench workload (host route assembly vs kernel calls).

    python tools/profile_route_build.py
"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from openr_amd import hiprt

    hiprt.set_device(0)
    dev = bench.Dev(0, 1)
    wl = bench.FacadeRouteBuild("fabric_lfa_routes", 0, 1, dev, None, None)
    wl.step()
    pr = cProfile.Profile()
    pr.enable()
    wl.step()
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(35)
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    from openr_amd.engine import close_all

    close_all()


if __name__ == "__main__":
    main()
