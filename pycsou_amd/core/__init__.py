from .linop import LinearOperator
from .functional import Functional, DifferentiableFunctional, ProximableFunctional, LinearFunctional
from .map import Map, DifferentiableMap
from .solver import GenericIterativeAlgorithm
