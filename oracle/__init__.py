"""TEST INFRASTRUCTURE ONLY: CPU restatement of the volkit reference serial path (parity
oracle and CPU baseline).  Never imported by the volkit_amd package."""
