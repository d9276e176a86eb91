import numpy as np

e = np.e
inf = np.inf
nan = np.nan
newaxis = None
pi = np.pi
