"""Drop-in replacement of the reference's ``FastMarching`` package (src/FastMarching/).

``import FastMarching.FastMarching as FM`` / ``import FastMarching.FastMarching3D as FM3D``
(Coupled_motion_planner.py:13-14) resolve here when ``planning-motion_planning_amd/`` is on
``sys.path`` ahead of the reference's ``src/``.  The solves and path extraction run on the
MI355X through libeikonal.so (include/eikonal.h); there is no CPU solver behind them.
"""
