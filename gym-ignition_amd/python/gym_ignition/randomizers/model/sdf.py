"""Randomized model descriptions (reference:
python/gym_ignition/randomizers/model/sdf.py): XPath-selected numeric
elements of a model file are resampled on every `sample()`.

Same builder API and semantics as the reference's SDFRandomizer
(Absolute / Additive / Coefficient methods, Uniform / Gaussian
distributions -- the Gaussian's `variance` field is used as the scale, as
the reference does --, `force_positive` clips the SAMPLE at zero,
`ignore_zeros` skips elements whose nominal value is 0, multi-match XPaths
expand to one randomization per element).  Differences: the standard
library's ElementTree replaces lxml (not installed here), and the model may
be the URDF itself -- this backend loads URDF directly, there is no
sdformat URDF->SDF conversion -- so a value is read from the element text
(SDF `<mass>1.0</mass>`) or, when the element has none, from its `value`
attribute (URDF `<mass value="1.0"/>`).  An SDF-style XPath such as
"*/link/inertial/mass" (the model level under <sdf>) also matches a URDF,
whose <robot> root is the model level.
"""

from enum import Enum, auto
from pathlib import Path
from typing import Dict, List, NamedTuple, Union
from xml.etree import ElementTree as etree

import numpy as np


class Distribution(Enum):
    Uniform = auto()
    Gaussian = auto()


class Method(Enum):
    Absolute = auto()
    Additive = auto()
    Coefficient = auto()


class GaussianParams(NamedTuple):
    variance: float
    mean: float = None


class UniformParams(NamedTuple):
    low: float
    high: float


DistributionParameters = Union[UniformParams, GaussianParams]


class RandomizationData(NamedTuple):
    xpath: str
    distribution: Distribution
    parameters: DistributionParameters
    method: Method
    ignore_zeros: bool = False
    force_positive: bool = False
    element: etree.Element = None


class RandomizationDataBuilder:
    """Chained construction of one randomization (reference builder API)."""

    def __init__(self, randomizer: "SDFRandomizer"):
        self.storage: Dict = {}
        self.randomizer = randomizer

    def at_xpath(self, xpath: str) -> "RandomizationDataBuilder":
        self.storage["xpath"] = xpath
        return self

    def sampled_from(self, distribution: Distribution,
                     parameters: DistributionParameters) -> "RandomizationDataBuilder":
        expected = GaussianParams if distribution is Distribution.Gaussian else UniformParams
        if not isinstance(parameters, expected):
            raise ValueError("Wrong parameters type")
        self.storage["distribution"] = distribution
        self.storage["parameters"] = parameters
        return self

    def method(self, method: Method) -> "RandomizationDataBuilder":
        self.storage["method"] = method
        return self

    def ignore_zeros(self, ignore_zeros: bool) -> "RandomizationDataBuilder":
        self.storage["ignore_zeros"] = ignore_zeros
        return self

    def force_positive(self, force_positive: bool = True) -> "RandomizationDataBuilder":
        self.storage["force_positive"] = force_positive
        return self

    def add(self) -> None:
        data = RandomizationData(**self.storage)
        if len(self.randomizer.find_xpath(data.xpath)) == 0:
            raise RuntimeError(f"Failed to find element matching XPath '{data.xpath}'")
        self.randomizer.insert(randomization_data=data)


class SDFRandomizer:
    """Randomized model-description generator over a model file (SDF or URDF)."""

    def __init__(self, sdf_model: str):
        self._sdf_file = sdf_model
        if not Path(self._sdf_file).is_file():
            raise ValueError(f"File '{sdf_model}' does not exist")
        self._root: etree.Element = etree.parse(self._sdf_file).getroot()
        self._randomizations: List[RandomizationData] = []
        self._default_values: Dict[etree.Element, float] = {}
        self.rng = np.random.default_rng()

    def seed(self, seed: int) -> None:
        self.rng = np.random.default_rng(seed)

    def find_xpath(self, xpath: str) -> List[etree.Element]:
        found = self._root.findall(xpath)
        if not found and self._root.tag == "robot" and xpath.startswith("*/"):
            found = self._root.findall(xpath[2:])  # URDF: <robot> is the model level
        return found

    def process_data(self) -> None:
        expanded = []
        for data in self._randomizations:
            elements = self.find_xpath(data.xpath)
            if len(elements) == 0:
                raise RuntimeError(f"Failed to find elements from XPath '{data.xpath}'")
            for element in elements:
                if data.ignore_zeros and self._value(element) == 0.0:
                    continue
                if data.method in (Method.Additive, Method.Coefficient):
                    self._default_values[element] = self._value(element)
                expanded.append(data._replace(element=element))
        self._randomizations = expanded

    def sample(self, pretty_print: bool = False) -> str:
        for data in self._randomizations:
            if data.distribution is Distribution.Gaussian:
                sample = self.rng.normal(loc=data.parameters.mean, scale=data.parameters.variance)
            elif data.distribution is Distribution.Uniform:
                sample = self.rng.uniform(low=data.parameters.low, high=data.parameters.high)
            else:
                raise ValueError("Distribution not recognized")
            if data.force_positive:
                sample = max(sample, 0.0)
            if data.method is Method.Absolute:
                value = sample
            elif data.method is Method.Additive:
                value = sample + self._default_values[data.element]
            elif data.method is Method.Coefficient:
                value = sample * self._default_values[data.element]
            else:
                raise ValueError("Method not recognized")
            self._set_value(data.element, value)
        if pretty_print:
            etree.indent(self._root)
        return etree.tostring(self._root, encoding="unicode")

    def new_randomization(self) -> RandomizationDataBuilder:
        return RandomizationDataBuilder(randomizer=self)

    def insert(self, randomization_data) -> None:
        self._randomizations.append(randomization_data)

    def get_active_randomizations(self) -> List[RandomizationData]:
        return self._randomizations

    def clean(self) -> None:
        self._randomizations = []
        self._default_values = {}
        self._root = etree.parse(self._sdf_file).getroot()

    @staticmethod
    def _value(element: etree.Element) -> float:
        text = (element.text or "").strip()
        if text:
            return float(text)
        if "value" in element.attrib:
            return float(element.attrib["value"])
        raise RuntimeError(f"The element {element.tag} does not have any content")

    @staticmethod
    def _set_value(element: etree.Element, value: float) -> None:
        if (element.text or "").strip() or "value" not in element.attrib:
            element.text = str(value)
        else:
            element.attrib["value"] = str(value)
