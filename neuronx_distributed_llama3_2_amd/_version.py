__version__ = "0.9.0+mi355x.r1"
