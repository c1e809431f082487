"""Test-infrastructure oracle package (CPU restatement of the reference step). Never on the product path."""
